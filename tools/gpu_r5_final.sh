#!/bin/bash
# Round 5 closing run on the final kernels: PMC traffic of the tail launch, the default bench
# (with the CPU baseline), its kernel-trace summary, the whole GPU suite, smoke.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fs gpurun_out/prof_final gpurun_out/summary.txt
mkdir -p gpurun_out/pmc_fs
run fs_plain 300 python -u tools/pmc_fused.py --self gpurun_out/pmc_fs/alg.json
run fs_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fs/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_f.json
run fs_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fs/write -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_w.json
python tools/pmc_summarize.py fused_block_s gpurun_out/pmc_fs gpurun_out/r05_pmc_fused_block_s.json > gpurun_out/pmc_fs.txt 2>&1
mkdir -p profiles && cp gpurun_out/r05_pmc_fused_block_s.json profiles/ 2>/dev/null
run final_bench 420 python -u bench.py
run final_bench_prof 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --parity-steps 1
run final_gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider
run final_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
