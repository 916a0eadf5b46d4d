#!/bin/bash
# round 6: C5 end-to-end line (generate vs codec decode split, gemm_f32_kernel roofline), its
# rocprof kernel summary, and the codec's MFMA-busy PMC pass at 32 x 751 frames (44.1 kHz head)
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
export CODEC=44k SHAPES=32x751
run c5_codec 300 python3 -u tools/bench_codec.py
run c5_bench 600 python3 -u bench.py --e2e --steps 2 --warmup 1
run c5_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python3 -u bench.py --e2e --steps 1 --warmup 1
# keep the summaries only (the per-launch trace of a whole generate is hundreds of MB)
find gpurun_out/prof_c5 -name '*kernel_trace.csv' -delete
du -sh gpurun_out/prof_c5 >> gpurun_out/summary.txt
run c5_pmc 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_c5 -o pmc --output-format csv -- python3 -u tools/bench_codec.py
du -sh gpurun_out/pmc_c5 >> gpurun_out/summary.txt
