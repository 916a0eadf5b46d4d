# Full GPU check: numerics tests, smoke, bench (+CPU baseline), rocprof kernel stats,
# PMC traffic of the gate/up launch. Usage: tools/gpucall.sh tools/gpu_round.sh 1500
source tools/gpu_run.sh
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py
run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
