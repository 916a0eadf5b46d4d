#!/bin/bash
# Round 6 closing checks: the whole GPU suite (its full-depth report -> gpurun_out/parity_full.json,
# the noise floor -> gpurun_out/noise_floor.json), then smoke
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6_full_gpu_tests.log 2>&1
rc=$?; echo "gpu suite rc=$rc" >> gpurun_out/r6_full_gpu_tests.log
tail -3 gpurun_out/r6_full_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_full_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r6_full_smoke.log; exit $rc
