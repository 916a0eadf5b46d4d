# Decode determinism at 12 / 16 rows: current library, then the session-start attention kernels.
source tools/gpu_run.sh
export TMPDIR=/tmp
run det 400 python -u tools/diag_fused_det.py 8 12,16
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_oldattn.so run det_oldattn 400 python -u tools/diag_fused_det.py 8 12,16
