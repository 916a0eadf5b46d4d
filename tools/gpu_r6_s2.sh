#!/bin/bash
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run bench_c3 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
run bench_c3p10 400 python -u bench.py --workload c3p10 --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
