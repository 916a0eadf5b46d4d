# Gate/up PMC passes only (FETCH_SIZE, WRITE_SIZE in separate runs) for the decode gate/up kernel.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gu
run gu_time 120 python3 tools/pmc_gateup.py
run gu_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gu/fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run gu_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_gu/write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
for d in pmc_gu/fetch pmc_gu/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py gate_up gpurun_out/pmc_gu gpurun_out/r02_pmc_gate_up.json > gpurun_out/pmc_gu.txt 2>&1
rm -f gpurun_out/pmc_gu/*/*counter_collection.csv
