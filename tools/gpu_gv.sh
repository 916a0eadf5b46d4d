# GEMV decode gate/up probe: micro timings, GEMV tests, bench default vs T5G_GU_GEMV=1
source tools/gpu_run.sh
export TMPDIR=/tmp
run micro_gemv 300 python -u tools/micro_gemv.py 8
run t_gemv 300 python -u -m pytest tests/test_gpu_gemv.py -q --timeout 120 --timeout-method thread
run bench_def 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
T5G_GU_GEMV=1 run bench_gu 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline
