#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s15_exact 600 python -u -m pytest -q --timeout 400 --timeout-method thread tests/test_gpu_exact.py
run s15_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s15_tiny 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sort_emu.py tests/test_gpu_sampler.py
run s15_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
