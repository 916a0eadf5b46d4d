# Multi-block sampler block timeline (diagnostic library).
source tools/gpu_run.sh
export TMPDIR=/tmp
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag_samp 300 python tools/diag_sampler.py
