# Iteration check: every GPU test, smoke, C3 bench + step timeline, C5 bench + step timeline.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
run t_gpu 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 700 python bench.py --no-cpu-baseline
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
rm -rf gpurun_out/prof_e2e
run prof_e2e 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e -o run --output-format csv -- python3 bench.py --e2e --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof_e2e/run_kernel_trace.csv > gpurun_out/trace_e2e.txt 2>&1
rm -f gpurun_out/prof_e2e/run_kernel_trace.csv
