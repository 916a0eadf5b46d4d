source tools/gpu_run.sh
export TMPDIR=/tmp
run tl_pf0 60 tools/bin/micro_timeline 527 0 1 0
run tl_pf64 60 tools/bin/micro_timeline 527 0 1 64
run tl_pf128 60 tools/bin/micro_timeline 527 0 1 128
run tl_pf256 60 tools/bin/micro_timeline 527 0 1 256
