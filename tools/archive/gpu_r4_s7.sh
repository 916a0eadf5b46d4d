#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s7_exact 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_exact.py -k "xmm"
run s7_probe 300 python -u tools/probe_xmm.py 1,8 var
run s7_parity 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "batch8_exact or golden_c2-32"
run s7_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
run s7_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
