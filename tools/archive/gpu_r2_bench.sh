# Round-2 measurement: C3 bench (+ measured CPU baseline), C5 e2e bench, rocprof kernel
# trace of one bench step reduced to a per-decode-step timeline.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
run t_ckpt 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_checkpoint.py
run bench 900 python -u bench.py
run bench_e2e 900 python -u bench.py --e2e --steps 2 --warmup 1
run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null
rm -f gpurun_out/prof/run_kernel_trace.csv
