# Probe: resid_norm launches with extra blocks that read the next GEMM's weights
# (T5G_NORM_PF=1) vs without; bench + per-step kernel timeline for both.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof0 gpurun_out/prof1
for m in 1 0; do
  export T5G_NORM_PF=$m
  run bench_pf$m 500 python bench.py --no-cpu-baseline
  run prof_pf$m 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$m -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  python tools/trace_step.py gpurun_out/prof$m/run_kernel_trace.csv > gpurun_out/trace_pf$m.txt 2>&1
  rm -f gpurun_out/prof$m/run_kernel_trace.csv
done
