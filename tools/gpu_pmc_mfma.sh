#!/bin/bash
# MFMA-pipe utilisation and effective clock per kernel of one bench meta-step (one --pmc pass,
# separate from any tracing). Summarise with tools/pmc_mfma_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing ${BENCH_ARGS:-}"
timeout -s KILL 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "${PMC_REGEX:-k_}" -f csv -d gpurun_out/pmc_mfma -o run -- python bench.py $BA \
  > gpurun_out/pmc_mfma.log 2>&1
echo "pmc_mfma rc=$?"
