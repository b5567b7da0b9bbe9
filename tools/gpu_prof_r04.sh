#!/bin/bash
# Round-4 profile of bench.py at HEAD for one per-rank workload (TASKS tasks on the GPU: 15 = the N=1
# meta-batch, 8 / 4 / 2 = rank 0's round-robin share at N = 2 / 4 / 8): kernel trace + stats, then separate
# rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (never combined with tracing). Output dir
# gpurun_out/prof_t$TASKS/ in the layout tools/prof_summary.py reads. Each pass has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TASKS:-15}
D=gpurun_out/prof_t$T
mkdir -p $D
KT="--tasks $T --steps 2 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $D/prof_kt -o run -- python bench.py $KT > $D/prof_kt.log 2>&1 || exit $?
echo "t$T kernel-trace ok"
PB="--tasks $T --steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 --no-timing"
RX="${PMC_REGEX:-k_lstm_fwd|k_lstm_bwd|k_wgrad|k_gcn_layer|k_gcn_mlp|k_gemm_nn}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d $D/prof_pmc_$C -o run -- python bench.py $PB > $D/prof_pmc_$C.log 2>&1 || exit $?
  echo "t$T pmc $C ok"
done
