# Probe (recorded in profiles/r02_probe_qkv_rx.txt): qkv projection on the split-K register-X GEMV
# (T5G_QKV_RX=1, a switch removed from engine.hip after this run) vs the tiled GEMM.
# C3 and C5 benches and the C3 step timeline for both.
source tools/gpu_run.sh
export TMPDIR=/tmp
for m in 1 0; do
  export T5G_QKV_RX=$m
  run bench_q$m 500 python bench.py --no-cpu-baseline
  run e2e_q$m 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
  rm -rf gpurun_out/profq$m
  run prof_q$m 500 rocprofv3 --kernel-trace --stats -d gpurun_out/profq$m -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
  python tools/trace_step.py gpurun_out/profq$m/run_kernel_trace.csv > gpurun_out/trace_q$m.txt 2>&1
  rm -f gpurun_out/profq$m/run_kernel_trace.csv
done
