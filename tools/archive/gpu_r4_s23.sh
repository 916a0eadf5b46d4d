#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s23_attn 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_fused.py
run s23_bench 400 python -u bench.py --no-cpu-baseline --parity-steps 0 --steps 3 --warmup 1
run s23_bench_noflash 400 python -u bench.py --no-cpu-baseline --parity-steps 0 --steps 3 --warmup 1 --no-attn-flash
run s23_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s23_prof -o run -- python -u bench.py --no-cpu-baseline --parity-steps 0 --steps 1 --warmup 0
run s23_full 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_parity_full.py -k "full_depth_batch8"
