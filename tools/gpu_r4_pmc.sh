#!/bin/bash
# HBM traffic per launch of the fast path's dominant kernel (fused_block_kernel, M = 8, C3
# shape) from PMC counters: separate FETCH_SIZE / WRITE_SIZE passes, no trace domains.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fb
run fb_plain 300 python -u tools/pmc_fused.py
run fb_fetch 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fb/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py
run fb_write 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fb/write -o pmc --output-format csv -- python3 tools/pmc_fused.py
for d in pmc_fb/fetch pmc_fb/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py fused_block gpurun_out/pmc_fb gpurun_out/r04_pmc_fused_block.json > gpurun_out/pmc_fb.txt 2>&1
tail -1 gpurun_out/fb_plain.log >> gpurun_out/summary.txt
