# Fused launch vs per-op launches, bitwise, at 1 / 8 / 12 / 16 / 32 rows.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_fused 600 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread
