# LDS prefill GEMM with an XCD-aware tile order vs the register ring (bitwise equal) at 480 / 1216 / 4864 tokens.
source tools/gpu_run.sh
export TMPDIR=/tmp
run pfx 300 python tools/probe_pf_lds.py
