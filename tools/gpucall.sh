#!/bin/bash
# usage: tools/gpucall.sh <script> [timeout]  -- clears local logs, runs the script on the GPU box
rm -f gpurun_out/summary.txt
timeout 2400 /usr/local/graft/bin/gpurun --timeout ${2:-1200} -- "bash $1" > /tmp/gpucall.out 2>&1
rc=$?
grep -E "^\[gpurun\] status|transient|refused" /tmp/gpucall.out | head -3
cat gpurun_out/summary.txt 2>/dev/null
exit $rc
