# Last-row difference: logits diagnostic with the register-ring prefill GEMM (diagnostic lib).
source tools/gpu_run.sh
export TMPDIR=/tmp
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_pfreg.so run detl_pfreg 500 python -u tools/diag_det_logits.py 6 16,12
run detl 500 python -u tools/diag_det_logits.py 6 16,12
