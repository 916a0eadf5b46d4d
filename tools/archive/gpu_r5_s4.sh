# round 5 session 4: glibc expf restated -- exact attention kernels, every parity golden
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  tests/test_gpu_exact.py \
  "tests/test_gpu_parity_full.py::test_sliding_window_long_prompt_golden" \
  "tests/test_gpu_parity_full.py::test_config_golden_exact" > gpurun_out/r5_s4_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5_s4_tests.log
grep -E "PASSED|FAILED|rows_bitwise|logit_rows_equal" gpurun_out/r5_s4_tests.log | tail -30
