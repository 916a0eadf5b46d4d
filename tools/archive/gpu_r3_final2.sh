# Round-3 closing measurement pass: every workload line, the rocprof trace of the default
# run, the fused-block timeline (diagnostic build) and the per-op unit timelines.
source tools/gpu_r3_final.sh
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python tools/diag_fused.py 8
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag_blocks 400 python tools/diag_blocks.py
