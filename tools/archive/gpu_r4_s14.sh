#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s14_lp4 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_parity_full.py -k "longprompt"
bash tools/gpu_r4_pmc.sh
run s14_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s14_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
run s14_bench 600 python -u bench.py
