#!/bin/bash
# Round-4 final profiles: tools/gpu_prof_r04.sh for the N=1 meta-batch (15 tasks) and rank 0's shares at
# N = 2 / 4 / 8 (8 / 4 / 2 tasks), then the MFMA / SQ PMC passes of the 15-task run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for T in 15 8 4 2; do
  TASKS=$T bash tools/gpu_prof_r04.sh || exit $?
done
D=gpurun_out/prof_t15
PB="--steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 --no-timing"
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA \
  --kernel-include-regex "k_lstm|k_wgrad|k_gcn" -f csv -d $D/prof_pmc_sq -o run -- python bench.py $PB > $D/prof_pmc_sq.log 2>&1 || exit $?
echo "sq pmc ok"
