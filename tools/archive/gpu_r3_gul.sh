# Gate/up unit in LDS (LDS-DMA during O1 -> O): bitwise fused-vs-unfused, c3 / c2 bench, block timeline.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_fused 600 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_fused.log || exit 1
run bench_c3 300 python -u bench.py --no-cpu-baseline
run bench_c2 300 python -u bench.py --workload c2 --no-cpu-baseline --steps 2
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python tools/diag_fused.py 8
