# round 5 session 5: parity-mode persistent layer (xlayer.hip) -- bitwise vs per-op, goldens, bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xlayer.py \
  > gpurun_out/r5_s5_xlayer.log 2>&1
rc=$?; echo "xlayer rc=$rc" >> gpurun_out/r5_s5_xlayer.log
grep -E "PASSED|FAILED|Error|error" gpurun_out/r5_s5_xlayer.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity_full.py::test_config_golden_exact" tests/test_gpu_exact.py > gpurun_out/r5_s5_goldens.log 2>&1
rc=$?; echo "goldens rc=$rc" >> gpurun_out/r5_s5_goldens.log
grep -E "PASSED|FAILED" gpurun_out/r5_s5_goldens.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --parity-steps 2 > gpurun_out/r5_s5_bench.log 2>&1
rc=$?; tail -c 3000 gpurun_out/r5_s5_bench.log; exit $rc
