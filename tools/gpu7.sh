source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run t_all 1200 python -m pytest tests -m gpu -q -x -s
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py
run dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 0 --dist-backend gloo --no-cpu-baseline
