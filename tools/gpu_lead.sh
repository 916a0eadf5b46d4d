# PRO_LEAD probe: GPU tests (lead gate/up by default), bench per site mask, per-step trace
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_lead4 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
T5G_LEAD_NORM=0 run bench_lead0 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
T5G_LEAD_NORM=7 run bench_lead7 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
rm -rf gpurun_out/prof_lead
run prof_lead 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lead -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof_lead/run_kernel_trace.csv > gpurun_out/trace_lead.txt 2>&1
rm -f gpurun_out/prof_lead/run_kernel_trace.csv
