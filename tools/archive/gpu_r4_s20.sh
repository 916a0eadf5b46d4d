#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s20_exact 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "decode_attention or attention_bitwise"
