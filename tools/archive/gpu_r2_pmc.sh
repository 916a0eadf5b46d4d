# HBM traffic per launch from PMC counters (separate FETCH_SIZE / WRITE_SIZE passes, no
# trace domains): decode gate/up GEMV and decode self attention.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gu gpurun_out/pmc_attn
run gu_plain 300 python -u tools/pmc_gateup.py
run gu_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gu/fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run gu_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_gu/write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run at_plain 300 python -u tools/pmc_attention.py
run at_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_attn/fetch -o pmc --output-format csv -- python3 tools/pmc_attention.py
run at_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_attn/write -o pmc --output-format csv -- python3 tools/pmc_attention.py
for d in pmc_gu/fetch pmc_gu/write pmc_attn/fetch pmc_attn/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py gate_up gpurun_out/pmc_gu gpurun_out/r02_pmc_gate_up.json > gpurun_out/pmc_gu.txt 2>&1
python tools/pmc_summarize.py attention gpurun_out/pmc_attn gpurun_out/r02_pmc_attention.json > gpurun_out/pmc_attn.txt 2>&1
tail -1 gpurun_out/gu_plain.log >> gpurun_out/summary.txt
tail -1 gpurun_out/at_plain.log >> gpurun_out/summary.txt
