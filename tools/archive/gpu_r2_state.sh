# Round-2 first check: GPU tests with printed parity rates (-s) + one bench line.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread
run bench 600 python bench.py --no-cpu-baseline
