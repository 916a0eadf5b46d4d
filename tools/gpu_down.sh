# Probe: decode down projection on gemv_dec split-K (T5G_DOWN_GEMV=1) vs the default gemm_p16.
source tools/gpu_run.sh
export TMPDIR=/tmp
run smoke_dg 300 env T5G_DOWN_GEMV=1 python -c "import __graft_entry__ as g; g.smoke()"
run t_dg 600 env T5G_DOWN_GEMV=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread
run bench_def 600 python bench.py --no-cpu-baseline
run bench_dg 600 env T5G_DOWN_GEMV=1 python bench.py --no-cpu-baseline
