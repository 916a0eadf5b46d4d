source tools/gpu_run.sh
rm -rf gpurun_out/summary.txt
export TMPDIR=/tmp
run micro_kernels 300 ./tools/bin/micro_kernels
