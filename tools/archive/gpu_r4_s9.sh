#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s9_exact 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_exact.py -k "xmm"
run s9_probe 300 python -u tools/probe_xmm.py 1,8 var
run s9_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
