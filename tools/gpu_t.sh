source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
