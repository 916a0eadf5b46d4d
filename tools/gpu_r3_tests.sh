# Full GPU test suite (one process), then smoke().
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
