source tools/gpu_run.sh
export TMPDIR=/tmp
T5G_LIB=$PWD/t5gemma-tts_amd/lib/libt5gtts_dbg.so run diag 300 python -u tools/diag_sampler.py
run t_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
