# Register-resident-X decode GEMV: numerics vs fp32 and vs the LDS-staged kernel, timing.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_rx 300 python -u -m pytest tests/test_gpu_gemv.py -v -x --timeout 200 --timeout-method thread
run sweep32 300 python tools/sweep_gate_up.py --m32
