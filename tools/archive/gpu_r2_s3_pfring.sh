# Probe: prefill GEMM register ring depth S = 2 / 4 / 6 / 8 (one library per depth).
# (tools/bin is listed in .gpurunignore since this ran: drop that line to run it again)
source tools/gpu_run.sh
export TMPDIR=/tmp
for S in 2 4 6 8; do
  T5G_LIB=$PWD/tools/bin/libt5gtts_pf$S.so run pf$S 120 python tools/probe_pf_stages.py
done
cat gpurun_out/pf*.log | grep lib > gpurun_out/probe_pf_stages.jsonl
