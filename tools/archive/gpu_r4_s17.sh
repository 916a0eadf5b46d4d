#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s17_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s17_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
