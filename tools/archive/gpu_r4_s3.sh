#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s3_parity 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_exact.py tests/test_gpu_parity_full.py tests/test_gpu_sampler.py tests/test_gpu_noise.py -k "not long"
run s3_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
run s3_bench_c2_parity 400 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 --warmup 1
run s3_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3_prof -o run -- python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 0
find gpurun_out/s3_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/s3_kernel_stats.csv
