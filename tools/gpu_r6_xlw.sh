#!/bin/bash
# round 6: the parity layer launch's Infinity Cache warm-up (xlayer.hip)
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xlw_probe 400 python3 -u tools/probe_xl_warm.py
run xlw_tests 600 python -u -m pytest tests/test_gpu_xlayer.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
