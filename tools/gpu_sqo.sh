# Probe: k-slices of the decode qkv (T5G_S_QKV) and o / cross-q / cross-o (T5G_S_O) projections.
source tools/gpu_run.sh
export TMPDIR=/tmp
run smoke_q4 300 env T5G_S_QKV=4 T5G_S_O=2 python -c "import __graft_entry__ as g; g.smoke()"
run bench_def 600 python bench.py --no-cpu-baseline
run bench_q4 600 env T5G_S_QKV=4 python bench.py --no-cpu-baseline
run bench_o2 600 env T5G_S_O=2 python bench.py --no-cpu-baseline
