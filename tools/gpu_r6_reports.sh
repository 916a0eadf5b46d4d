#!/bin/bash
# round 6 closing: the full-depth report and the noise floor on the final fast-path sources
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt gpurun_out/noise_floor_progress.txt
run reports 900 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_noise_floor.py -x -v -s --timeout 880 --timeout-method thread -p no:cacheprovider
