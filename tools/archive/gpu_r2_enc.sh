# XCodec2 encoder + codec decoder + CLI / pipeline GPU tests.
source tools/gpu_run.sh
export TMPDIR=/tmp
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
run t_enc 600 $T tests/test_gpu_codec_enc.py tests/test_gpu_codec.py tests/test_gpu_cli.py tests/test_gpu_pipeline.py
grep -E "passed|failed|error|features max" gpurun_out/t_enc.log | tail -6 >> gpurun_out/summary.txt
