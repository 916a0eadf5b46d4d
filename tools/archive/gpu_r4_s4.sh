#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s4_mm4 120 bash -c "hipcc -O3 -Wno-unused-result --offload-arch=gfx950 tools/micro_mfma4.hip -o /tmp/mm4 && /tmp/mm4"
run s4_probe 300 python -u tools/probe_xmm.py 1,8,32
run s4_pfl 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_prefill_lds.py
run s4_sampler 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sampler.py tests/test_gpu_noise.py tests/test_gpu_pipeline.py
run s4_bench_c3_parity 400 python -u bench.py --workload c3 --parity --no-cpu-baseline --steps 1 --warmup 1
