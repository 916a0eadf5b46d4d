source tools/gpu_run.sh
export TMPDIR=/tmp
run diag 200 python -u tools/diag_cli_whisper.py
