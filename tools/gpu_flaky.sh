# Repeat the GPU parity tests to measure flakiness (sequential, one process each).
source tools/gpu_run.sh
export TMPDIR=/tmp
for i in 1 2 3 4; do
  run t_gpu_$i 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread
done
