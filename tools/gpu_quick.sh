# Quick GPU iteration: GPU tests + bench without CPU baseline.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 900 python bench.py --no-cpu-baseline
