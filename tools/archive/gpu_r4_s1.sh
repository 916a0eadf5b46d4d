#!/bin/bash
# round 4 step 1: device MT19937 noise + device tie order + chunked parity loop; xmm linear
source tools/gpu_run.sh
export TMPDIR=/tmp
run s1_xmm 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "linear"
run s1_noise 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_noise.py tests/test_gpu_sampler.py
run s1_parity 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_exact.py tests/test_gpu_parity_full.py -k "not long and not linear"
run s1_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
run s1_bench_c2_parity 400 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1 --warmup 1
