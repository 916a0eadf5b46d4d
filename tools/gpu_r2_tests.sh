# Round-2 GPU test pass: full -m gpu suite with printed parity rates.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 1500 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
