# stage S at the end of the previous launch (attn_in_block 2): bitwise vs the flash launch, then
# the bench in modes 2 / 1 / 0
mkdir -p gpurun_out
rm -f gpurun_out/r5_s28_*
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_attn_in_block.py \
  > gpurun_out/r5_s28_attn_in_block.log 2>&1
rc=$?; echo "attn_in_block rc=$rc" >> gpurun_out/r5_s28_attn_in_block.log
grep -E "PASSED|FAILED|Error|error" gpurun_out/r5_s28_attn_in_block.log | tail -14
[ $rc -eq 0 ] || exit $rc
for m in 2 1; do
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 --attn-in-block $m > gpurun_out/r5_s28_bench_m$m.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s28_bench_m$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 --no-attn-in-block > gpurun_out/r5_s28_bench_m0.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s28_bench_m0.log | cut -c1-200; exit $rc
