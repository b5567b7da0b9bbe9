#!/bin/bash
# Round-3 profile of the default bench at HEAD: kernel trace + stats, then separate rocprofv3 --pmc
# passes (FETCH_SIZE, WRITE_SIZE, MFMA busy, SQ instruction mix). SMAML_COOP=0 (the default since): the grid-barrier
# kernels are launched with a plain launch of the same grid (rocprofv3 crashed in its exit handlers
# after hipLaunchCooperativeKernel). Each pass has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp SMAML_COOP=0
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt -o run -- python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 > gpurun_out/prof_kt.log 2>&1 || exit $?
echo "kernel-trace ok"
PB="--steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --no-timing"
RX="${PMC_REGEX:-k_lstm_fwd|k_lstm_bwd|k_wgrad|k_gcn_layer|k_gcn_mlp|k_gemm_nn}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d gpurun_out/prof_pmc_$C -o run -- python bench.py $PB > gpurun_out/prof_pmc_$C.log 2>&1 || exit $?
  echo "pmc $C ok"
done
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_mfma -o run -- python bench.py $PB > gpurun_out/pmc_mfma.log 2>&1 || exit $?
echo "pmc mfma ok"
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_sq -o run -- python bench.py $PB > gpurun_out/pmc_sq.log 2>&1 || exit $?
echo "pmc sq ok"
