#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s28_c2 300 python -u bench.py --workload c2 --no-cpu-baseline --parity-steps 0
run s28_c2_parity 300 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 --warmup 1
run s28_c4 300 python -u bench.py --workload c4 --no-cpu-baseline --parity-steps 0
run s28_c5 400 python -u bench.py --e2e --no-cpu-baseline --parity-steps 0
