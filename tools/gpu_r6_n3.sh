#!/bin/bash
# round 6: N3 inside the 17-32-row MLP-half launch -- fused / attention GPU tests, the C5
# end-to-end line and its rocprof kernel summary
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run n3_tests 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_attn_in_block.py
run n3_bench 600 python3 -u bench.py --e2e --steps 2 --warmup 1
run n3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n3 -o c5 --output-format csv -- python3 -u bench.py --e2e --steps 1 --warmup 1
find gpurun_out/prof_n3 -name '*kernel_trace.csv' -delete
