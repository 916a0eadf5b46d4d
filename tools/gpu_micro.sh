# Kernel micro-benchmarks (fused GEMV sweep) + GEMV numerics + engine parity + short bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gemv 300 python -u -m pytest tests/test_gpu_gemv.py -q --timeout 120 --timeout-method thread
run micro_gemv 300 python -u tools/micro_gemv.py 8
run t_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 900 python bench.py --no-cpu-baseline --steps 2
