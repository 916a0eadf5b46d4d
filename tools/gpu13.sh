source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
run micro_kernels 300 ./tools/bin/micro_kernels
run t_parity 900 python -m pytest tests/test_gpu_parity.py -q -x
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run bench 900 python bench.py --no-cpu-baseline
