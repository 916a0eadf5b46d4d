# round 5 session 1: the window diagnosis + the capacity / codec-at-size / hygiene tests
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u tools/dbg/dbg_window_kv.py gpu > gpurun_out/r5_s1_window_kv.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_attention.py tests/test_gpu_exact.py \
  "tests/test_gpu_parity_full.py::test_fast_path_capacity_is_per_call" \
  "tests/test_gpu_parity_full.py::test_sliding_window_long_prompt_golden" \
  "tests/test_gpu_codec.py::test_c5_codec_44k_at_size" > gpurun_out/r5_s1_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5_s1_tests.log
tail -5 gpurun_out/r5_s1_tests.log
