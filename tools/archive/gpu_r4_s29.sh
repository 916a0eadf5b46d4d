#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s29_eager_kernel 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_eager.py -k bitwise
run s29_eager_golden 600 python -u -m pytest -v -s --timeout 500 --timeout-method thread tests/test_gpu_eager.py -k golden
