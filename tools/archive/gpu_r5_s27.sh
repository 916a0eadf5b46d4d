# fast path: decode self attention as stage S of the persistent layer launch -- bitwise vs the
# flash launch, the fused / attention suites, then the bench with and without it
mkdir -p gpurun_out
rm -f gpurun_out/r5_s27_*
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_attn_in_block.py \
  > gpurun_out/r5_s27_attn_in_block.log 2>&1
rc=$?; echo "attn_in_block rc=$rc" >> gpurun_out/r5_s27_attn_in_block.log
grep -E "PASSED|FAILED|Error|error" gpurun_out/r5_s27_attn_in_block.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_attention.py > gpurun_out/r5_s27_fused_attn.log 2>&1
rc=$?; echo "fused/attention rc=$rc" >> gpurun_out/r5_s27_fused_attn.log
grep -cE "PASSED" gpurun_out/r5_s27_fused_attn.log; grep -E "FAILED|rc=" gpurun_out/r5_s27_fused_attn.log | tail -5
[ $rc -eq 0 ] || exit $rc
FS_VARS=0,0,5 timeout -k 10 300 python -u tools/diag_fused_s.py 8 376 > gpurun_out/r5_s27_diag_s.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5_s27_diag_s.log | sed -n '/rep 1 variant 0/,/rep 2/p'; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 > gpurun_out/r5_s27_bench_on.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s27_bench_on.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 --no-attn-in-block \
  > gpurun_out/r5_s27_bench_off.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s27_bench_off.log | cut -c1-600; exit $rc
