#!/bin/bash
# HBM traffic per call of the fast path's flash decode self attention (attn_decode_kernel
# FLASH, C3 shape) from PMC counters: separate FETCH_SIZE / WRITE_SIZE passes, no trace domains.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_at
run at_plain 300 python -u tools/pmc_attention.py --flash
run at_fetch 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_at/fetch -o pmc --output-format csv -- python3 tools/pmc_attention.py --flash
run at_write 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_at/write -o pmc --output-format csv -- python3 tools/pmc_attention.py --flash
for d in pmc_at/fetch pmc_at/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py attention_flash gpurun_out/pmc_at gpurun_out/r04_pmc_attention_flash.json > gpurun_out/pmc_at.txt 2>&1
tail -1 gpurun_out/at_plain.log >> gpurun_out/summary.txt
