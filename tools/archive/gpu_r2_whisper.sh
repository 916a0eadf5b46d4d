# Whisper recognizer GPU tests (parity vs transformers goldens, transcribe control flow).
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_whisper 600 python -u -m pytest tests/test_gpu_whisper.py -v -s -x --timeout 300 --timeout-method thread
run b_whisper 300 python tools/bench_whisper.py --seconds 10 --iters 5
run p_whisper 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wh -o run --output-format csv -- python3 tools/bench_whisper.py --seconds 10 --iters 2
