#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s30_c3_parity_eager 500 python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 1
run s30_c3_fast_eager 400 python -u bench.py --attn eager --no-cpu-baseline --parity-steps 0
run s30_c2_parity_eager 500 python -u bench.py --workload c2 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 1
run s30_prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s30_prof -o run -- python -u bench.py --workload c3 --parity --attn eager --no-cpu-baseline --steps 1 --warmup 0
