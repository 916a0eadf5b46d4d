mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py -x -v --timeout 500 --timeout-method thread -k "longprompt or sliding_window" > gpurun_out/r4_4k.log 2>&1
