#!/bin/bash
# PMC traffic of the tail launch (fused_block_kernel<2>) at the bench rows' final length, then
# the default bench line that prices it
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fs gpurun_out/summary.txt
mkdir -p gpurun_out/pmc_fs
run fs_plain 300 python -u tools/pmc_fused.py --self gpurun_out/pmc_fs/alg.json
run fs_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fs/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_f.json
run fs_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fs/write -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_w.json
python tools/pmc_summarize.py fused_block_s gpurun_out/pmc_fs gpurun_out/r05_pmc_fused_block_s.json > gpurun_out/pmc_fs.txt 2>&1
cp gpurun_out/r05_pmc_fused_block_s.json profiles/ 2>/dev/null
run final_bench2 420 python -u bench.py
