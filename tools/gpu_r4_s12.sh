#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s12_cache 300 python -u tools/dbg/dbg_cache_hash.py gpu golden_longprompt
run s12_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
