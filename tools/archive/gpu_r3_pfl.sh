# LDS-staged prefill GEMM: ring depth A/B (NBUF 2 / 3 / 4) at 2 waves per SIMD, bitwise vs the register ring.
source tools/gpu_run.sh
export TMPDIR=/tmp
run pfl3 300 python tools/probe_pf_lds.py
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_pfl2.so run pfl2 300 python tools/probe_pf_lds.py
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_pfl4.so run pfl4 300 python tools/probe_pf_lds.py
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python tools/diag_fused.py 8
