source tools/gpu_run.sh
export TMPDIR=/tmp
run tlb 120 tools/bin/micro_tlb
