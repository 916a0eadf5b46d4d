source tools/gpu_run.sh
export TMPDIR=/tmp
run sweep32 300 python tools/sweep_gate_up.py --m32
