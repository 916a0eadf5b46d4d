# Kernel trace of one C5 (B = 32) end-to-end bench step, reduced per decode step.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof_e2e
run prof_e2e 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e -o run --output-format csv -- python3 bench.py --e2e --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof_e2e/run_kernel_trace.csv > gpurun_out/trace_e2e.txt 2>&1
rm -f gpurun_out/prof_e2e/run_kernel_trace.csv
