# Where the rare last-row difference starts (logits of every step, host loop).
source tools/gpu_run.sh
export TMPDIR=/tmp
run detl 500 python -u tools/diag_det_logits.py 6 16,12
