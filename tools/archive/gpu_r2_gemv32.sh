# 17..32-row decode GEMV: numerics, batch invariance, C5 end-to-end bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gemv 400 python -u -m pytest tests/test_gpu_gemv.py "tests/test_gpu_parity.py::test_batch32_rows_equal_single_rows" "tests/test_gpu_parity.py::test_batched_rows_equal_single_rows" -v -x --timeout 300 --timeout-method thread
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
