#!/bin/bash
# Round 4: phase probe of the small-grid kernels (probe build), then the headline A/B of the
# weight-gradient / tangent-BPTT knobs (k_wgrad_ws with 8 producer waves; pair-segment tile order)
# with PMC passes. Every GPU step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in "12 12" "0 0" "3 1"; do
  set -- $p
  timeout -k 10 240 python -u tools/kw_probe.py --diag $1 --bdiag $2 >> gpurun_out/r04j_probe.log 2>&1 || exit $?
done
cat gpurun_out/r04j_probe.log | grep -v Warn | tail -30
timeout -k 10 900 python -u tools/ab_run.py gpurun_out/r04j_ab.log 1 base=libsmaml.so ws=libsmaml.so:SMAML_OPTIONS=wgrad_ws=1 \
  remap=libsmaml.so:SMAML_OPTIONS=bwdd_remap=1 || exit $?
BA="--steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing --adapt-epochs 0 --cfg5-share-tasks 0"
SMAML_OPTIONS=wgrad_ws=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_wgrad" -f csv -d gpurun_out/r04j_pmc_ws -o run -- python bench.py $BA > gpurun_out/r04j_pmc_ws.log 2>&1
r=$?; echo "pmc rc=$r"; [ $r -eq 0 ] || exit $r
for v in off:bwdd_remap=0 on:bwdd_remap=1; do
  n=${v%%:*}; o=${v#*:}
  SMAML_OPTIONS=$o timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_lstm_bwd_dual" -f csv -d gpurun_out/r04j_fetch_$n -o run -- python bench.py $BA > gpurun_out/r04j_fetch_$n.log 2>&1
  r=$?; echo "fetch $n rc=$r"; [ $r -eq 0 ] || exit $r
done
