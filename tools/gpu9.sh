source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run t_sampler 600 python -m pytest tests/test_gpu_sampler.py -q -x -s
run t_parity 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -q -x -s
run micro_sampler 300 python tools/micro_sampler.py
run bench 900 python bench.py --no-cpu-baseline
