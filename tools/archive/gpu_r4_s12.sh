#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s12_cache 300 python -u tools/dbg/dbg_cache_hash.py gpu golden_longprompt
run s12_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s12_tiny 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_exact.py
run s12_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
