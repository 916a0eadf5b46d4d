# Round-2 kernel iteration: attention + engine parity tests, then the C3 bench (no CPU
# baseline) and a rocprof per-step timeline.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
run t_attn 600 $T tests/test_gpu_attention.py tests/test_gpu_parity.py tests/test_gpu_parity_full.py tests/test_gpu_checkpoint.py
run bench 600 python -u bench.py --no-cpu-baseline
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null
rm -f gpurun_out/prof/run_kernel_trace.csv
grep -E "passed|failed|error" gpurun_out/t_attn.log | tail -3 >> gpurun_out/summary.txt
