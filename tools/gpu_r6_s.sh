#!/bin/bash
# round 6: stage S past 1 024 keys -- bitwise tests, then the C3 and 10 s-prompt C3 lines
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run s_tests 900 python -u -m pytest tests/test_gpu_attn_in_block.py tests/test_gpu_fused.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/s_tests.log && ! grep -q "FAILED\| failed" gpurun_out/s_tests.log || exit 1
run bench_c3 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
run bench_c3p10 400 python -u bench.py --workload c3p10 --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0
