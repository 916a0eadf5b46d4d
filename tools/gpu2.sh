source tools/gpu_run.sh
rm -f gpurun_out/summary.txt
run t_tiny 600 python -m pytest tests/test_gpu_parity.py -q -s -k "tiny or batched or graph"
run t_mid 600 python -m pytest tests/test_gpu_parity.py -q -s -k "mid"
