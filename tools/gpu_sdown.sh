# Probe: k-slices of the decode down projection (T5G_S_DOWN) -- GEMM spread vs slab bytes the norm reads.
source tools/gpu_run.sh
export TMPDIR=/tmp
run smoke_s4 300 env T5G_S_DOWN=4 python -c "import __graft_entry__ as g; g.smoke()"
run bench_s8 600 python bench.py --no-cpu-baseline
run bench_s4 600 env T5G_S_DOWN=4 python bench.py --no-cpu-baseline
run bench_s6 600 env T5G_S_DOWN=6 python bench.py --no-cpu-baseline
