#!/bin/bash
# round 6: what Infinity-Cache-resident weights would buy the layer launches
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run probe_mall 400 python3 -u tools/probe_mall_layer.py
