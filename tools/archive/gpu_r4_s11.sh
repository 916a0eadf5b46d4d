#!/bin/bash
source tools/gpu_run.sh
export TMPDIR=/tmp
run s11_cache 300 python -u tools/dbg/dbg_cache_hash.py gpu golden_longprompt
