# Bench after the register-ring prefill switch: C3 (default, with CPU baseline) and C5 e2e.
source tools/gpu_run.sh
export TMPDIR=/tmp
run bench_c3 700 python bench.py
run bench_c5 500 python bench.py --e2e --steps 2 --warmup 1 --no-cpu-baseline
run bench_c2 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 2
