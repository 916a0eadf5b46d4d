source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run micro_kernels 300 ./tools/bin/micro_kernels
run t_parity 900 python -m pytest tests/test_gpu_parity.py -q -x
run bench 900 python bench.py --no-cpu-baseline
