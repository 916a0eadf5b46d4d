# MFMA utilisation of the MFMA-bound kernels (one PMC pass, no trace domains).
source tools/gpu_run.sh
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_mfma
run mfma_plain 300 python -u tools/pmc_mfma_driver.py
run mfma_pmc 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o pmc --output-format csv -- python3 tools/pmc_mfma_driver.py
f=$(ls gpurun_out/pmc_mfma/*counter_collection.csv 2>/dev/null | head -1)
[ -n "$f" ] && python tools/pmc_mfma.py "$f" gpurun_out/r03_pmc_mfma.json > gpurun_out/pmc_mfma.txt 2>&1
rm -f gpurun_out/pmc_mfma/*counter_collection.csv
