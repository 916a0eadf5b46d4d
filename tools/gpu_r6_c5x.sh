#!/bin/bash
# round 6: cross attention sized by the call's text bound -- attention / fused GPU tests, the
# C5 end-to-end line and its rocprof kernel summary
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run c5x_tests 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_attention.py tests/test_gpu_attn_in_block.py
run c5x_bench 600 python3 -u bench.py --e2e --steps 2 --warmup 1
run c5x_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5x -o c5 --output-format csv -- python3 -u bench.py --e2e --steps 1 --warmup 1
find gpurun_out/prof_c5x -name '*kernel_trace.csv' -delete
