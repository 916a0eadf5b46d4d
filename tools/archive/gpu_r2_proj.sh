source tools/gpu_run.sh
export TMPDIR=/tmp
run sweep_proj 300 python tools/sweep_proj.py
