# Session-3 closing measurements: GPU tests, smoke, C3 bench (with CPU baseline), C5 bench,
# rocprof kernel stats + step timeline, PMC HBM traffic of gate/up and attention.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_gu gpurun_out/pmc_attn
run t_gpu 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 700 python bench.py
run e2e 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_default.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
run gu_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gu/fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run gu_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_gu/write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run at_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_attn/fetch -o pmc --output-format csv -- python3 tools/pmc_attention.py
run at_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_attn/write -o pmc --output-format csv -- python3 tools/pmc_attention.py
for d in pmc_gu/fetch pmc_gu/write pmc_attn/fetch pmc_attn/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py gate_up gpurun_out/pmc_gu gpurun_out/r02_pmc_gate_up.json > gpurun_out/pmc_gu.txt 2>&1
python tools/pmc_summarize.py attention gpurun_out/pmc_attn gpurun_out/r02_pmc_attention.json > gpurun_out/pmc_attn.txt 2>&1
rm -f gpurun_out/pmc_gu/*/*counter_collection.csv gpurun_out/pmc_attn/*/*counter_collection.csv
