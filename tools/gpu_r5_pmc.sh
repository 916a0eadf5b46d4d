#!/bin/bash
# Round 5: HBM traffic per launch of the parity path's dominant kernel (xlayer_kernel, M = 8,
# C3 shape) from PMC counters (separate FETCH_SIZE / WRITE_SIZE passes, no trace domains), and
# the kernel-trace summary of the default bench command.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_xl gpurun_out/prof_bench
run xl_plain 300 python -u tools/pmc_xlayer.py
run xl_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_xl/fetch -o pmc --output-format csv -- python3 tools/pmc_xlayer.py
run xl_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_xl/write -o pmc --output-format csv -- python3 tools/pmc_xlayer.py
for d in pmc_xl/fetch pmc_xl/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py xlayer gpurun_out/pmc_xl gpurun_out/r05_pmc_xlayer.json > gpurun_out/pmc_xl.txt 2>&1
run bench_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --parity-steps 1
tail -2 gpurun_out/xl_plain.log >> gpurun_out/summary.txt
