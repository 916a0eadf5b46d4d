#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s27_exact 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_parity.py
run s27_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s27_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
run s27_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s27_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
