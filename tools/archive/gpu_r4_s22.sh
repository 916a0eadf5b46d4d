#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s22_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s22_tiny 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_exact.py
run s22_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
run s22_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s22_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
