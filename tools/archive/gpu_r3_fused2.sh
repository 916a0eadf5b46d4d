# Fused decode MLP half: bitwise test, block timeline, C3 bench, kernel trace.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof_f
run t_fused 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread
grep -q " passed" gpurun_out/t_fused.log || exit 1
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python tools/diag_fused.py 8
run bench_f 400 python bench.py --no-cpu-baseline
run prof_f 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof_f/run_kernel_trace.csv > gpurun_out/trace_fused.txt 2>&1
cp gpurun_out/prof_f/run_kernel_stats.csv gpurun_out/kernel_stats_fused.csv 2>/dev/null
rm -f gpurun_out/prof_f/run_kernel_trace.csv
