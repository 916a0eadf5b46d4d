#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s13_cache 300 python -u tools/dbg/dbg_cache_hash.py gpu golden_longprompt
run s13_parity 900 python -u -m pytest -v --timeout 800 --timeout-method thread tests/test_gpu_parity_full.py -k "config_golden or batch8_exact"
run s13_gpu_a 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_exact.py tests/test_gpu_prefill_lds.py tests/test_gpu_fused.py tests/test_gpu_distributed.py
run s13_det 400 python -u tools/diag_det_logits.py 4 16,12
