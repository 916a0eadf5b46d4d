# Round-2 closing check of the committed tree: every GPU test (parity rates printed),
# smoke, default bench (with CPU baseline), C5 end-to-end bench, rocprof kernel stats and
# per-step timeline of one bench generate().
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
run t_gpu 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 700 python bench.py
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
