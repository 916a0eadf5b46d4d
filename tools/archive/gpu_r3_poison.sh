# Fused launch: bitwise vs per-op at 1-32 rows, and the hand-off timeout fallback.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_fused 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread
