source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
export TMPDIR=/tmp
run t_all 900 python -m pytest tests/test_gpu_parity.py -q -s
run micro_sampler 300 python tools/micro_sampler.py
run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
run bench 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline
