#!/bin/bash
# Stall / occupancy / cache diagnosis of the LSTM kernels on one task group of the config-2 bench
# (5 tasks = one group, 1 meta-step): separate --pmc passes (never combined with tracing), each
# under its own time limit. Summarise with tools/pmc_diag_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BA="--tasks 5 --steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing ${BENCH_ARGS:-}"
RX="${PMC_REGEX:-k_lstm_bwd|k_lstm_fwd|k_wgrad<}"
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
         "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE" ${PMC_EXTRA:-}; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-include-regex "$RX" -f csv -d gpurun_out/pmc_diag_$i -o run -- \
    python bench.py $BA > gpurun_out/pmc_diag_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
