source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run micro_kernels 300 ./tools/bin/micro_kernels
run t_parity 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_sampler.py -q -x
run exp_groups 900 python tools/exp_groups.py
