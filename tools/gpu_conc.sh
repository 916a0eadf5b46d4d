source tools/gpu_run.sh
export TMPDIR=/tmp
run conc 120 tools/bin/micro_concurrency
