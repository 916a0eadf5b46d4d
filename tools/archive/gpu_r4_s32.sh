#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s32_eager 700 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_eager.py
run s32_c3_parity_eager 500 python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 1
run s32_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s32_prof -o run -- python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 0
