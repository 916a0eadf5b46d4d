#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s16_exact 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "xmm"
run s16_probe 300 python -u tools/probe_xmm.py 1,8 var
run s16_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s16_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
