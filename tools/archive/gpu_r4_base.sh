#!/bin/bash
# round 4 baseline: C3 parity bench + rocprof kernel stats of the parity run
source tools/gpu_run.sh
export TMPDIR=/tmp
run r4b_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
run r4b_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
find gpurun_out/r4b_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/r4b_kernel_stats.csv
