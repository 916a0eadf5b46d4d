#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s2_dbg 300 python -u tools/dbg/dbg_parity_graph.py
run s2_xmm 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "linear"
run s2_exact_tiny 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_exact.py -k "tiny or attention"
