# Sampler: one-batch row-state reads. Sampler tests, c3 bench, rocprof trace of the step.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_samp 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_samp.log || exit 1
grep -q "failed" gpurun_out/t_samp.log && exit 1
run bench_c3 300 python -u bench.py --no-cpu-baseline
rm -rf gpurun_out/prof
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
