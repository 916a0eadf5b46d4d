source tools/gpu_run.sh
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run bench 900 python bench.py --no-cpu-baseline --steps 2
