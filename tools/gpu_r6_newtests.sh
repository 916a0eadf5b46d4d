#!/bin/bash
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run new_tests 900 python -u -m pytest tests/test_gpu_attn_in_block.py tests/test_gpu_codec.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider
