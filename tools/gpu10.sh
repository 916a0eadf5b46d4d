source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run micro_kernels 300 ./tools/bin/micro_kernels
run t_sampler 600 python -m pytest tests/test_gpu_sampler.py -q -x -s
run micro_sampler 300 python tools/micro_sampler.py
