#!/bin/bash
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
hipcc -O3 --offload-arch=gfx950 tools/micro_graph_fork.hip -o /tmp/gf > gpurun_out/gf_build.log 2>&1 || exit 1
run gf 60 /tmp/gf
