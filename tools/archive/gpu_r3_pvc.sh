# P.V/combine: scores + chunk maxima requested before V. Attention tests, c3 bench, block timelines.
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_attn 600 python -u -m pytest tests/test_gpu_attention.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_attn.log || exit 1
grep -q "failed" gpurun_out/t_attn.log && exit 1
run bench_c3 300 python -u bench.py --no-cpu-baseline
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag_blocks 400 python tools/diag_blocks.py
