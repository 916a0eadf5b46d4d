# Parity-mode attention with up-front K / V requests: exact tests + C2 parity bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_exact 600 python -u -m pytest tests/test_gpu_exact.py -x -q --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_exact.log || exit 1
run bench_c2_parity 300 python -u bench.py --workload c2 --parity --no-cpu-baseline --steps 1
