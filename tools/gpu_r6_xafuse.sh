#!/bin/bash
# round 6: the parity decode attention's scores + P.V as one launch (xattn_fused_kernel)
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xaf_tests 700 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_xlayer.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/xaf_tests.log && ! grep -q "FAILED\| failed" gpurun_out/xaf_tests.log || exit 1
run xaf_prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_xaf -o xa --output-format csv -- python3 -u bench.py --parity --steps 1 --warmup 1 --no-cpu-baseline
find gpurun_out/prof_xaf -name '*kernel_trace.csv' -delete
