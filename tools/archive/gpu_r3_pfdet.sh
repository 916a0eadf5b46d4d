# Run-to-run determinism of the prefill GEMMs.
source tools/gpu_run.sh
export TMPDIR=/tmp
run pfdet 300 python tools/probe_pf_det.py
