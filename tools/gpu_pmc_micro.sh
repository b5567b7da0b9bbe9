#!/bin/bash
# SQ / TA counter passes over tools/gate_micro (one rocprofv3 run per pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM" \
           "${PMC3:-TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET -f csv -d gpurun_out/pmc_micro$i -o run -- ./tools/gate_micro > gpurun_out/pmc_micro$i.log 2>&1
  echo "pass $i rc=$?"
done
