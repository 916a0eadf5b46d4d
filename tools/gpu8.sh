source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
run micro_latency 120 ./tools/bin/micro_latency
run gateup 300 python tools/pmc_gateup.py
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python3 tools/pmc_gateup.py
run bench 900 python bench.py --no-cpu-baseline
