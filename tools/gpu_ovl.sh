source tools/gpu_run.sh
export TMPDIR=/tmp
run ovl256 60 tools/bin/micro_overlap 256
run ovl512 60 tools/bin/micro_overlap 512
