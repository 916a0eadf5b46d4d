source tools/gpu_run.sh
export TMPDIR=/tmp
run t_cli 400 python -u -m pytest tests/test_gpu_cli.py -v -x -s --timeout 300 --timeout-method thread
