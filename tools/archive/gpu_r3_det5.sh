# Last-row difference: the LDS prefill GEMM with its tail requests into a spare stage.
source tools/gpu_run.sh
export TMPDIR=/tmp
run detl 500 python -u tools/diag_det_logits.py 6 16,12
run pfdet 300 python -u tools/probe_pf_det.py
