#!/bin/bash
# round 6: the consumer-norm persistent exact layer -- bitwise tests, goldens, parity bench
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xl_tests 300 python -u -m pytest tests/test_gpu_xlayer.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider
grep -q "passed" gpurun_out/xl_tests.log && grep -q " 0 failed\|passed in" gpurun_out/xl_tests.log || exit 1
run xl_goldens 600 python -u -m pytest tests/test_gpu_exact.py -k "engine" tests/test_gpu_parity_full.py -k "engine or exact or golden" -x -v --timeout 500 --timeout-method thread -p no:cacheprovider
run xl_bench 400 python -u bench.py --parity --steps 2 --warmup 1 --no-cpu-baseline
