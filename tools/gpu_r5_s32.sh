# fast path cross-attention stage: LDS-only barriers, VALU exchanges, wave-0 publish -- bitwise
# tests (fused vs per-op, stage S, eager fast path), then the bench
mkdir -p gpurun_out
rm -f gpurun_out/r5_s32_*
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_attn_in_block.py "tests/test_gpu_eager.py::test_eager_fast_path" > gpurun_out/r5_s32_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_s32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 > gpurun_out/r5_s32_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s32_bench.log | cut -c1-130; exit $rc
