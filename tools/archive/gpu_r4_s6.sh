#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s6_exact 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_exact.py -k "xmm"
run s6_probe 300 python -u tools/probe_xmm.py 1,8 var
run s6_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s6_prof -o probe -- python -u tools/probe_xmm.py 8
run s6_parity 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "batch8_exact or config_golden"
run s6_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
