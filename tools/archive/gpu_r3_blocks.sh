# Block timelines of the per-op units (self-attention scores / P.V, head, sampler).
source tools/gpu_run.sh
export TMPDIR=/tmp
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag_blocks 400 python tools/diag_blocks.py
