# dx kernel adopted for K = 2304 split GEMMs at 17..32 rows: GEMM tests, engine parity,
# head GEMM probe, C5 bench + timeline.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof5
run t_gemm 300 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 120 --timeout-method thread -k "gemm or batch32 or batched"
run head 200 python tools/probe_head.py
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run prof5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run --output-format csv -- python3 bench.py --e2e --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof5/run_kernel_trace.csv > gpurun_out/trace_c5.txt 2>&1
rm -f gpurun_out/prof5/run_kernel_trace.csv
