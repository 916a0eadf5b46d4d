set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/xlayer_timeline.py > gpurun_out/r06_base_xlayer_timeline.log 2>&1 && \
timeout -k 10 400 python -u bench.py --parity --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r06_base_parity.log 2>&1
