#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run r04f_gpu_tests 1100 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread
