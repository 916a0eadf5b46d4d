source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt gpurun_out/prof_codec
export TMPDIR=/tmp
run t_codec 600 python -m pytest tests/test_gpu_codec.py -q -s -x
run bench_codec 300 python tools/bench_codec.py
run prof_codec 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_codec -o run --output-format csv -- python3 tools/bench_codec.py
