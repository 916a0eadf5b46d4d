# round 5 session 2: capacity / codec-at-size / hygiene tests after the ABI cap fix
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_attention.py tests/test_gpu_exact.py \
  "tests/test_gpu_parity_full.py::test_fast_path_capacity_is_per_call" \
  "tests/test_gpu_parity_full.py::test_sliding_window_long_prompt_golden" \
  "tests/test_gpu_codec.py::test_c5_codec_44k_at_size" > gpurun_out/r5_s2_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5_s2_tests.log
tail -15 gpurun_out/r5_s2_tests.log
