#!/bin/bash
# Final-build evidence: SQ instruction mix pass on the config-2 bench, then the config-4 adaptation
# A/B (default vs f32 MFMA build) with its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_sq -o run -- python bench.py --steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing > gpurun_out/pmc_sq.log 2>&1 || exit $?
python tools/pmc_sq_summary.py gpurun_out/pmc_sq > gpurun_out/pmc_sq.txt 2>&1
head -8 gpurun_out/pmc_sq.txt
TESTS= AB_VARIANTS="libsmaml_f32.so" AB_ROUNDS=1 bash tools/gpu_ab_adapt.sh
