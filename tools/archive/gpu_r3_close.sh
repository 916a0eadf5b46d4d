# Closing checks: full GPU suite and smoke() on the tree, decode determinism at 12 / 16 rows
# (engine prefill on the register ring), and the spare-stage LDS prefill variant (diagnostic lib).
source tools/gpu_run.sh
export TMPDIR=/tmp
run t_gpu 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rxX
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run detl 400 python -u tools/diag_det_logits.py 6 16,12
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_spare.so run detl_spare 400 python -u tools/diag_det_logits.py 6 16,12
