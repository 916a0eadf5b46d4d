#!/bin/bash
# Round 6 closing: the whole GPU suite and smoke on the final tree, then the default bench line
mkdir -p gpurun_out
timeout -k 10 960 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6_closing_gpu_tests.log 2>&1
rc=$?; echo "gpu suite rc=$rc" >> gpurun_out/r6_closing_gpu_tests.log
tail -3 gpurun_out/r6_closing_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6_closing_smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r6_closing_bench.log 2>&1
rc=$?; tail -1 gpurun_out/r6_closing_bench.log | cut -c1-300; exit $rc
