# Block-level timelines of one decoder layer (diagnostic library): attention variants.
source tools/gpu_run.sh
export TMPDIR=/tmp
run tl_t0x1 120 tools/bin/micro_timeline 527 0 1
run tl_t1x1 120 tools/bin/micro_timeline 527 1 1
run tl_t1x4 120 tools/bin/micro_timeline 527 1 4
run tl_t0x4 120 tools/bin/micro_timeline 527 0 4
run tl_t1x4_200 120 tools/bin/micro_timeline 200 1 4
run t_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
