# Fused MLP checkpoint: all GPU tests, smoke, C3 bench (+CPU baseline), C5 e2e, kernel trace,
# PMC HBM bytes of the fused launch.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fm
run t_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 700 python bench.py
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/kernel_stats.csv 2>/dev/null
rm -f gpurun_out/prof/run_kernel_trace.csv
run fm_fetch 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fm/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py
run fm_write 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fm/write -o pmc --output-format csv -- python3 tools/pmc_fused.py
for d in pmc_fm/fetch pmc_fm/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && mv "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py fused_block gpurun_out/pmc_fm gpurun_out/r03_pmc_fused_block.json > gpurun_out/pmc_fm.txt 2>&1
