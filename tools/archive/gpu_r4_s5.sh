#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s5_exact 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_exact.py -k "xmm"
run s5_probe 300 python -u tools/probe_xmm.py 1,8,32
run s5_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
