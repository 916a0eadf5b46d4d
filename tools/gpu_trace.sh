# Per-step kernel timelines of the decode graph (default path and the fused-prologue P16 variant).
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof_*
trace() {  # name, T5G_FUSED_DECODE value
  export T5G_FUSED_DECODE=$2
  run prof_$1 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  python tools/trace_step.py gpurun_out/prof_$1/run_kernel_trace.csv > gpurun_out/trace_$1.txt 2>&1
  rm -f gpurun_out/prof_$1/run_kernel_trace.csv
}
trace default 0
trace fusedp16 2
