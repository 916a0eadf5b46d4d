# the other workloads on the closing kernels (tail stage S by default), after the stage-S tests
mkdir -p gpurun_out
rm -f gpurun_out/r5_other_*
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_attn_in_block.py tests/test_gpu_fused.py \
  > gpurun_out/r5_other_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r5_other_tests.log; [ $rc -eq 0 ] || exit $rc
for w in c2 c4; do
timeout -k 10 400 python -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --parity-steps 0 > gpurun_out/r5_other_$w.log 2>&1
rc=$?; tail -1 gpurun_out/r5_other_$w.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5_other_c5.log 2>&1
rc=$?; tail -1 gpurun_out/r5_other_c5.log | cut -c1-300; exit $rc
