# Probe: LDS-X shared decode GEMM (T5G_DX = row groups per block) vs default.
source tools/gpu_run.sh
export TMPDIR=/tmp
for m in 0 1 2 4; do
  T5G_DX=$m run dx$m 240 python tools/probe_dx.py
done
cat gpurun_out/dx*.log | grep '^{' > gpurun_out/probe_dx.jsonl
