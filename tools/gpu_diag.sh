source tools/gpu_run.sh
export TMPDIR=/tmp
run diag 300 python -u tools/diag_prefill.py
