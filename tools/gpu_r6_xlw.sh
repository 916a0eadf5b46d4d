#!/bin/bash
# round 6: which bytes' cache residency the parity layer launch is sensitive to
source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run xls_probe 400 python3 -u tools/probe_xl_share.py
