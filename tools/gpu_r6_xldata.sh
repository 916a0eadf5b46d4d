#!/bin/bash
# round 6: the parity layer's norm -> GEMV hand-offs by their data (xlayer.hip xl_wait_x16)
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xld_tests 700 python -u -m pytest tests/test_gpu_xlayer.py tests/test_gpu_parity.py tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/xld_tests.log && ! grep -q "FAILED\| failed" gpurun_out/xld_tests.log || exit 1
run xld_bench 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-steps 2
