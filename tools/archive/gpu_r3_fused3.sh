# Fused decode MLP half: bitwise test, block timeline, C3 bench.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_fused 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_fused.log || exit 1
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python tools/diag_fused.py 8
run bench_f 400 python bench.py --no-cpu-baseline
