#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s33_eager 700 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_gpu_eager.py tests/test_gpu_exact.py
run s33_c3_parity_eager 500 python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 1
