source tools/gpu_run.sh
export TMPDIR=/tmp
run diag 300 python -u tools/diag_prefill.py
run micro_prefill 300 python -u tools/micro_prefill.py
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
