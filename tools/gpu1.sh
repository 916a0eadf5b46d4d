set -o pipefail
cd $GRAFT_REPO_ROOT
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -s -k "gemm" > gpurun_out/t_gemm.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -s -k "sampler" > gpurun_out/t_sampler.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -s -k "tiny" > gpurun_out/t_tiny.log 2>&1
echo "exit $?"
