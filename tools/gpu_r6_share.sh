#!/bin/bash
# round 6: which bytes' cache residency the persistent layer launches are sensitive to
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run cache_share 400 python3 -u tools/probe_cache_share.py
