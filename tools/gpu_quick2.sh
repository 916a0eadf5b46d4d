source tools/gpu_run.sh
export TMPDIR=/tmp
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run t_gemv2 300 python -u -m pytest tests/test_gpu_gemv.py -q --timeout 120 --timeout-method thread
run t_gemv3 300 python -u -m pytest tests/test_gpu_gemv.py -q --timeout 120 --timeout-method thread
