#!/bin/bash
# round 6: the parity decode attention's P.V launch with every read up front
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xa_tests 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_xlayer.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/xa_tests.log && ! grep -q "FAILED\| failed" gpurun_out/xa_tests.log || exit 1
run xa_prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xa -o xa --output-format csv -- python3 -u bench.py --parity --steps 1 --warmup 1 --no-cpu-baseline
find gpurun_out/prof_xa -name '*kernel_trace.csv' -delete
