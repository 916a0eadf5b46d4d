# round 5 session 3: the 100 s-prompt golden, the CLI extremes, then the bench
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 800 --timeout-method thread \
  "tests/test_gpu_parity_full.py::test_config_golden_exact" \
  "tests/test_gpu_cli.py::test_run_inference_accepts_reference_extremes" > gpurun_out/r5_s3_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r5_s3_tests.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/r5_s3_bench.jsonl 2> gpurun_out/r5_s3_bench.err
echo "bench rc=$?" >> gpurun_out/r5_s3_tests.log
tail -12 gpurun_out/r5_s3_tests.log; tail -c 1500 gpurun_out/r5_s3_bench.jsonl
