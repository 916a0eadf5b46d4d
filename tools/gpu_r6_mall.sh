#!/bin/bash
# round 6: what Infinity-Cache-resident weights would buy the G stage and the layer launches
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I t5gemma-tts_amd/csrc tools/micro_gstage.hip -o /tmp/mg > gpurun_out/mg_build.log 2>&1 || exit 1
run mg_hbm 120 /tmp/mg 4
run mg_mall 120 /tmp/mg 1
run probe_mall 400 python3 -u tools/probe_mall_layer.py
