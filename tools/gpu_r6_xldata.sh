#!/bin/bash
# round 6: the parity layer's norm -> GEMV hand-offs by their data: timing + stage timeline
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xld_tests 400 python -u -m pytest tests/test_gpu_xlayer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/xld_tests.log && ! grep -q "FAILED\| failed" gpurun_out/xld_tests.log || exit 1
run xld_share 300 python3 -u tools/probe_cache_share.py
run xld_timeline 300 python -u tools/xlayer_timeline.py
