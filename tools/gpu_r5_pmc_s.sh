#!/bin/bash
# Round 5: HBM traffic per launch of the fast path's dominant kernel now that it carries the
# self attention (fused_block_kernel<true>, M = 8, C3 shape, ~527 keys) from PMC counters
# (separate FETCH_SIZE / WRITE_SIZE passes, no trace domains), and the kernel-trace summary of
# the default bench command.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fs gpurun_out/prof_bench_s gpurun_out/summary.txt
mkdir -p gpurun_out/pmc_fs
run fs_plain 300 python -u tools/pmc_fused.py --self gpurun_out/pmc_fs/alg.json
run fs_fetch 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fs/fetch -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_f.json
run fs_write 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fs/write -o pmc --output-format csv -- python3 tools/pmc_fused.py --self gpurun_out/pmc_fs/alg_w.json
for d in pmc_fs/fetch pmc_fs/write; do
  f=$(ls gpurun_out/$d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$d/pmc_counter_collection.csv
done
python tools/pmc_summarize.py fused_block_s gpurun_out/pmc_fs gpurun_out/r05_pmc_fused_block_s.json > gpurun_out/pmc_fs.txt 2>&1
[ -n "$NO_BENCH_PROF" ] && exit 0
run bench_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_s -o bench --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --parity-steps 1
tail -3 gpurun_out/fs_plain.log >> gpurun_out/summary.txt
tail -1 gpurun_out/bench_prof.log | cut -c1-300 >> gpurun_out/summary.txt
