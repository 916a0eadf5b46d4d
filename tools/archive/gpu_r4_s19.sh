#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s19_exact 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "decode_attention or attention_bitwise"
run s19_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s19_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
run s19_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s19_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
