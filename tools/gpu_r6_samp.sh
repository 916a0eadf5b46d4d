#!/bin/bash
# round 6: where the sampler's ~35 us per step go (block timeline, diagnostic library)
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run samp_micro 200 python3 -u tools/micro_sampler.py
export T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so
run samp_diag 200 python3 -u tools/diag_sampler.py
