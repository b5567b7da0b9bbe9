#!/bin/bash
# SQ counter passes (separate from any tracing) on the hot LSTM kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
RX="${PMC_REGEX:-lstm_fwd_step|lstm_bwd_step|k_wgrad|k_gemm_nn}"
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing --order 1 --tasks 15"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $SET --kernel-include-regex "$RX" -f csv -d gpurun_out/pmc_sq$i -o run -- python bench.py $BA > gpurun_out/pmc_sq$i.log 2>&1
  echo "set $i rc=$?"
done
