#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s10_exact 600 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_exact.py -k "602 or 603 or xmm"
run s10_probe 300 python -u tools/probe_xmm.py 1,8 var
run s10_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
