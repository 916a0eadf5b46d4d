#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s34_eager 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_eager.py
run s34_c3_parity_eager 500 python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 1
