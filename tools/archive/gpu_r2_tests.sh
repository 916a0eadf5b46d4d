# Round-2 GPU test pass: full -m gpu suite with printed parity rates.
source tools/gpu_run.sh
export TMPDIR=/tmp
(python -c "import torch; print('cpu capability', torch.backends.cpu.get_cpu_capability(), 'threads', torch.get_num_threads())"; lscpu | head -20) > gpurun_out/host_cpu.txt 2>&1
run t_gpu 1100 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread
