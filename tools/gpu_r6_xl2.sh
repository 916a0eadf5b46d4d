#!/bin/bash
# round 6 iteration: xlayer bitwise tests, stage timeline, parity bench
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xl_tests 300 python -u -m pytest tests/test_gpu_xlayer.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
grep -q "5 passed" gpurun_out/xl_tests.log || exit 1
run xl_timeline 300 python -u tools/xlayer_timeline.py
run xl_bench 400 python -u bench.py --parity --steps 2 --warmup 1 --no-cpu-baseline
