#!/bin/bash
# round 6: fp64 noise floor of the fast path (one C3 row, 100 steps), then the C3 and 10 s-prompt C3 lines
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt gpurun_out/noise_floor_progress.txt
run noise_floor 900 python -u -m pytest tests/test_gpu_noise_floor.py -x -v -s --timeout 880 --timeout-method thread -p no:cacheprovider
run bench_c3 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
run bench_c3p10 300 python -u bench.py --workload c3p10 --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
