#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run r04f_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run r04f_bench 600 python -u bench.py
run r04f_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_prof -o run -- python -u bench.py --no-cpu-baseline --parity-steps 0 --steps 1 --warmup 0
