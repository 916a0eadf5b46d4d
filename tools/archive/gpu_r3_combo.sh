# Parity attention check + the round-3 measurement pass in one call.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_exact 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_exact.log || exit 1
source tools/gpu_r3_final.sh
