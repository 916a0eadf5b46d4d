# A/B: Infinity-Cache warm-up of each decode layer's MLP weights (T5G_L3_WARM blocks).
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/prof
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
T5G_L3_WARM=128 run t_warm 300 $T tests/test_gpu_parity.py -k "tiny_engine or batched or graph"
for w in 0 64 128 256 0; do
  T5G_L3_WARM=$w run bench_w$w 300 python -u bench.py --no-cpu-baseline --steps 2
  tail -1 gpurun_out/bench_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('warm $w', d['value'], d['roofline']['decode_step_us'], d['roofline']['avg_us'])" >> gpurun_out/summary.txt
done
T5G_L3_WARM=128 run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python tools/trace_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/trace_warm.txt 2>&1
rm -f gpurun_out/prof/run_kernel_trace.csv
