# Round-3 measurement pass of the committed tree: every workload line + trace.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
run bench_c3 700 python bench.py
run bench_c2 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 2
run bench_c4 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 2
run bench_c5 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run bench_c2_parity 300 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1
run bench_c3_parity 400 python -u bench.py --parity --no-cpu-baseline --steps 1
run bench_c3_unfused 300 python -u bench.py --no-cpu-baseline --no-fused
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null
rm -f gpurun_out/prof/run_kernel_trace.csv
