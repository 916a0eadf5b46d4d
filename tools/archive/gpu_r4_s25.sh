#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s25_attn 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_fused.py
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run s25_diag 400 python -u tools/diag_flash.py
run s25_bench 400 python -u bench.py --no-cpu-baseline --parity-steps 0 --steps 3 --warmup 1
