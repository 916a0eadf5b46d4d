# Session-3 re-entry check of the committed tree: every GPU test, smoke, C3 bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 700 python bench.py
