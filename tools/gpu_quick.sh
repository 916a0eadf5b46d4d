# Quick GPU iteration: fused-GEMV numerics + engine parity + bench without CPU baseline.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gemv 300 python -u -m pytest tests/test_gpu_gemv.py -x -v --timeout 120 --timeout-method thread
run t_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 900 python bench.py --no-cpu-baseline
