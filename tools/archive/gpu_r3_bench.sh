#!/bin/bash
# round 3: bench lines for every workload + parity mode (run via gpurun)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py > gpurun_out/r3_bench_c3.json 2> gpurun_out/r3_bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 2 > gpurun_out/r3_bench_c2.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 2 > gpurun_out/r3_bench_c4.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 > gpurun_out/r3_bench_c2_parity.json 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --parity --no-cpu-baseline --steps 1 > gpurun_out/r3_bench_c3_parity.json 2>&1 || exit $?
tail -n 2 gpurun_out/r3_bench_*.json
