# xlayer: balanced G/D passes, parallel softmax p, shuffle tail of the sum of squares
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xlayer.py \
  > gpurun_out/r5_s11_xlayer.log 2>&1
rc=$?; echo "xlayer rc=$rc" >> gpurun_out/r5_s11_xlayer.log
grep -E "PASSED|FAILED|Error|error" gpurun_out/r5_s11_xlayer.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity_full.py::test_config_golden_exact" tests/test_gpu_exact.py > gpurun_out/r5_s11_goldens.log 2>&1
rc=$?; echo "goldens rc=$rc" >> gpurun_out/r5_s11_goldens.log
grep -cE "PASSED" gpurun_out/r5_s11_goldens.log; grep -E "FAILED|rc=" gpurun_out/r5_s11_goldens.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/xlayer_timeline.py 8 > gpurun_out/r5_s11_timeline.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r5_s11_timeline.log | sed -n '/rep 1 variant 0/,/rep 2/p'; exit $rc
