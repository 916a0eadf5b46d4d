# packed head-pair arithmetic in stage S: bitwise tests, then the bench in modes 2 / 0
mkdir -p gpurun_out
rm -f gpurun_out/r5_s31_*
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_attn_in_block.py \
  > gpurun_out/r5_s31_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_s31_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 2 0; do
if [ $m = 0 ]; then f=--no-attn-in-block; else f="--attn-in-block $m"; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-steps 0 $f > gpurun_out/r5_s31_bench_m$m.log 2>&1
rc=$?; tail -1 gpurun_out/r5_s31_bench_m$m.log | cut -c1-130; [ $rc -eq 0 ] || exit $rc
done
FS_VARS=0,0 timeout -k 10 300 python -u tools/diag_fused_s.py 8 376 > gpurun_out/r5_s31_diag.log 2>&1
grep -v amdgpu.ids gpurun_out/r5_s31_diag.log | sed -n '/rep 1 /,$p'
