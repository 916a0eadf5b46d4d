#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s18_c2_parity 400 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 --warmup 1
run s18_c2 400 python -u bench.py --workload c2 --no-cpu-baseline --parity-steps 0
run s18_c4 400 python -u bench.py --workload c4 --no-cpu-baseline --parity-steps 0
run s18_c5 600 python -u bench.py --workload c5 --no-cpu-baseline
