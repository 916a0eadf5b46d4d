# xlayer: pipelined GEMV stages -- bitwise tests, then the stage timeline
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xlayer.py \
  > gpurun_out/r5_s7_xlayer.log 2>&1
rc=$?; echo "xlayer rc=$rc" >> gpurun_out/r5_s7_xlayer.log
grep -E "PASSED|FAILED|Error|error" gpurun_out/r5_s7_xlayer.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/xlayer_timeline.py 8 > gpurun_out/r5_s7_timeline.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5_s7_timeline.log | tail -22; exit $rc
