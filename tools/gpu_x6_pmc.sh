#!/bin/bash
# PMC passes (MFMA busy / clock; SQ instruction mix) on one library, then a bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SMAML_LIB=weatherforecast_stgcn_maml_amd/${PMC_LIB:-libsmaml.so}
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_mfma -o run -- python bench.py $BA > gpurun_out/pmc_mfma.log 2>&1 || exit $?
python tools/pmc_mfma_summary.py gpurun_out/pmc_mfma > gpurun_out/pmc_mfma.txt 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_sq -o run -- python bench.py $BA > gpurun_out/pmc_sq.log 2>&1 || exit $?
unset SMAML_LIB
cat gpurun_out/pmc_mfma.txt | head -12
: > gpurun_out/ab.log
for round in 1 2; do
  for v in ${AB_VARIANTS}; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
python tools/ab_summary.py gpurun_out/ab.log
