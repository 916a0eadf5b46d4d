# Full GPU check: numerics tests, smoke, bench (+CPU baseline), rocprof kernel stats and
# per-step timeline, PMC traffic of the gate/up launch, layer block timeline.
# Usage: tools/gpucall.sh tools/gpu_round.sh 1500
source tools/gpu_run.sh
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py
run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run timeline 120 tools/bin/micro_timeline 527 0 1 0
