# Gate/up GEMV launch-shape sweep (waves, fragments in flight, block cap).
source tools/gpu_run.sh
export TMPDIR=/tmp
run sweep 300 python tools/sweep_gate_up.py
