# Round-end check of the committed tree: GPU tests, smoke, default bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py
