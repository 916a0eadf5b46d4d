#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s31_eager 700 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_gpu_eager.py
run s31_fused 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_attention.py
run s31_c3_fast_eager 400 python -u bench.py --attn eager --no-cpu-baseline --parity-steps 0
run s31_c3_fast 400 python -u bench.py --no-cpu-baseline --parity-steps 0
