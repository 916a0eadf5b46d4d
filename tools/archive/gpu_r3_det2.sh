# Fused tests (incl. the hand-off timeout fallback), then decode determinism at 12 / 16 rows:
# current library, the session-start attention kernels, and the single-block sampler.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_fused 600 python -u -m pytest tests/test_gpu_fused.py -v --timeout 300 --timeout-method thread
run det 400 python -u tools/diag_fused_det.py 8 12,16
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_oldattn.so run det_oldattn 400 python -u tools/diag_fused_det.py 8 12,16
DET_SAMPLER_SINGLE=1 run det_single 400 python -u tools/diag_fused_det.py 8 12,16
