source tools/gpu_run.sh
export TMPDIR=/tmp
run tl 60 tools/bin/micro_timeline 527 0 1 0
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
