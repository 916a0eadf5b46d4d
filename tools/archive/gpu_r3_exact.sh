#!/bin/bash
# round 3: exact-mode kernels -- bitwise tests, long goldens, parity C2 bench + kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py tests/test_gpu_parity_full.py tests/test_gpu_parity.py > gpurun_out/r3x_tests.log 2>&1 || { tail -30 gpurun_out/r3x_tests.log; exit 1; }
tail -3 gpurun_out/r3x_tests.log
timeout -k 10 300 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 > gpurun_out/r3x_bench_c2_parity.json 2>&1 || exit $?
tail -1 gpurun_out/r3x_bench_c2_parity.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3x_prof -o run -- python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/r3x_prof.log 2>&1 || exit $?
find gpurun_out/r3x_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/r3x_kernel_stats.csv
head -8 gpurun_out/r3x_kernel_stats.csv | cut -c1-200
