# Full GPU test suite (one process), then __graft_entry__.smoke().
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
