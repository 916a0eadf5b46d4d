# XCodec2 encoder timing (10 s prompt at 16 kHz dims) + kernel stats.
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof_enc
run enc_bench 300 python -u tools/bench_codec_enc.py --seconds 10 --iters 5
run enc_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_enc -o run --output-format csv -- python3 tools/bench_codec_enc.py --seconds 10 --iters 2
cp gpurun_out/prof_enc/run_kernel_stats.csv gpurun_out/enc_kernel_stats.csv 2>/dev/null
rm -f gpurun_out/prof_enc/run_kernel_trace.csv
tail -1 gpurun_out/enc_bench.log >> gpurun_out/summary.txt
