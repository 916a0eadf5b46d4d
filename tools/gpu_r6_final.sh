#!/bin/bash
# Round 6 closing measurement: fresh PMC passes (HBM bytes per launch) of the two dominant
# kernels on this tree's sources, then the default bench line that quotes them, then the
# rocprof kernel summary of the same command.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fs gpurun_out/pmc_xl gpurun_out/prof_final6 gpurun_out/summary.txt
mkdir -p gpurun_out/pmc_fs gpurun_out/pmc_xl
run fs_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fs/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_f.json
run fs_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fs/write -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_w.json
cp gpurun_out/pmc_fs/alg_f.json gpurun_out/pmc_fs/alg.json
run xl_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_xl/fetch -o pmc --output-format csv -- python3 tools/pmc_xlayer.py
run xl_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_xl/write -o pmc --output-format csv -- python3 tools/pmc_xlayer.py
for d in pmc_xl/fetch pmc_xl/write pmc_fs/fetch pmc_fs/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py fused_block_s gpurun_out/pmc_fs gpurun_out/r06_pmc_fused_block_s.json > gpurun_out/pmc_fs.txt 2>&1
python tools/pmc_summarize.py xlayer gpurun_out/pmc_xl gpurun_out/r06_pmc_xlayer.json > gpurun_out/pmc_xl.txt 2>&1
cp gpurun_out/r06_pmc_*.json profiles/ 2>/dev/null
run final_bench 600 python -u bench.py
run final_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final6 -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --parity-steps 1
find gpurun_out/prof_final6 -name '*kernel_trace.csv' -delete
