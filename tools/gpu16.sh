source tools/gpu_run.sh
export TMPDIR=/tmp
run t_parity 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_sampler.py tests/test_gpu_pipeline.py -q -x
run micro_kernels 300 ./tools/bin/micro_kernels
run micro_sampler 300 python tools/micro_sampler.py
run bench 900 python bench.py --no-cpu-baseline
