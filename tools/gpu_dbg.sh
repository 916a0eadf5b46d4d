source tools/gpu_run.sh
export TMPDIR=/tmp
export T5G_ATTN_TICKETS=0
run var_t0 300 python -u -m pytest tests/test_gpu_parity.py -k "variants or teacher" -v -s --timeout 120 --timeout-method thread
export T5G_ATTN_TICKETS=1
run var_t1 300 python -u -m pytest tests/test_gpu_parity.py -k "variants or teacher" -v -s --timeout 120 --timeout-method thread
