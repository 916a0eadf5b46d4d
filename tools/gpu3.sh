source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run t_all 900 python -m pytest tests/test_gpu_parity.py -q -s
run bench 900 python bench.py --steps 2 --warmup 1
