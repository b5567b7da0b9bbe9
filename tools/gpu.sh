#!/bin/bash
# The one runner for GPU-box sessions (replaces the per-session tools/gpu_*.sh scripts of rounds 1-4).
#
#   bash tools/gpu.sh STEP [STEP ...]
#
# Steps (run in order; the first crash-like exit -- fault, abort, segfault, time limit -- ends the
# session, a failed test run or bench ends it too; nothing is retried):
#   tests           python -m pytest tests -m gpu (PYTEST_K selects with -k, PYTEST_ARGS adds arguments)
#   smoke           __graft_entry__.smoke()
#   bench           python bench.py $BENCH_ARGS          -> gpurun_out/$TAG/bench.log (JSON line last)
#   prof            rocprofv3 --kernel-trace --stats of bench.py for one per-rank workload, then separate
#                   --pmc FETCH_SIZE / WRITE_SIZE passes     -> gpurun_out/$TAG/prof_t$TASKS[_c5]/
#                   (TASKS, default 15; CONFIG 2 or 5; tools/prof_summary.py reads the directory)
#   pmc_sq          SQ instruction-mix / MFMA-busy counters of the same workload (one --pmc pass)
#   pmc_clk         MFMA busy + effective clock (GRBM_GUI_ACTIVE) per kernel (tools/pmc_mfma_summary.py)
#   shares          one-GPU timings of rank 0's share at N = 2 / 4 / 8 (8 / 4 / 2 tasks)
#   ab              A/B: AB_VARIANTS (words "lib:<file in the package dir>", "opt:<k=v[,k=v]>" or both as
#                   "lib:<file>+opt:<k=v>", or "arg:<extra bench.py args, + for spaces>"; "base" =
#                   the default library) each in its own process, AB_ROUNDS interleaved rounds of
#                   bench.py $AB_ARGS                      -> gpurun_out/$TAG/ab.log
# TAG names the output directory (default "session").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-session}
O=gpurun_out/$TAG
mkdir -p "$O"
PKG=weatherforecast_stgcn_maml_amd

ok() {  # rc name: stop the session on anything but success
  local rc=$1
  echo "[$2] rc=$rc"
  [ "$rc" -eq 0 ] || exit "$rc"
}

bench_json() { grep '^{' "$1" | tail -1; }

workload_args() {  # per-rank workload of the prof / pmc steps
  local t=${TASKS:-15}
  if [ "${CONFIG:-2}" = 5 ]; then echo "--config 5 --tasks $t"; else echo "--tasks $t"; fi
}

for s in "$@"; do
  case $s in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
        -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > "$O/pytest_gpu.log" 2>&1
      rc=$?
      tail -3 "$O/pytest_gpu.log"
      ok $rc tests ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
      rc=$?
      tail -1 "$O/smoke.log"
      ok $rc smoke ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1
      rc=$?
      bench_json "$O/bench.log" | cut -c1-400
      ok $rc bench ;;
    prof)
      W=$(workload_args)
      D="$O/prof_t${TASKS:-15}$([ "${CONFIG:-2}" = 5 ] && echo _c5)"
      mkdir -p "$D"
      KT="$W --steps ${PROF_STEPS:-2} --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0"
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d "$D/prof_kt" -o run -- python bench.py $KT \
        > "$D/prof_kt.log" 2>&1
      ok $? prof_kt
      PB="$W --steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 --no-timing"
      RX="${PMC_REGEX:-k_lstm_fwd|k_lstm_bwd|k_wgrad|k_gcn_layer|k_gcn_mlp|k_gcn_expand|k_gcn_compact|k_gemm_nn|k_gemm_nt|k_xg|k_dg_rowsum}"
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 600 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d "$D/prof_pmc_$C" -o run -- \
          python bench.py $PB > "$D/prof_pmc_$C.log" 2>&1
        ok $? "pmc_$C"
      done ;;
    pmc_sq)
      W=$(workload_args)
      PB="$W --steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 --no-timing"
      timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_lstm|k_wgrad|k_gcn" \
        -f csv -d "$O/prof_pmc_sq" -o run -- python bench.py $PB > "$O/prof_pmc_sq.log" 2>&1
      ok $? pmc_sq ;;
    pmc_clk)
      # MFMA busy cycles and the effective clock (GRBM_GUI_ACTIVE / 8 over each dispatch's wall time)
      W=$(workload_args)
      PB="$W --steps 1 --warmup 0 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 --no-timing"
      timeout -s KILL 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
        --kernel-include-regex "k_lstm|k_wgrad|k_gcn|k_dg_rowsum|k_xg" -f csv -d "$O/prof_pmc_clk" -o run -- \
        python bench.py $PB > "$O/prof_pmc_clk.log" 2>&1
      ok $? pmc_clk ;;
    shares)
      : > "$O/shares.log"
      for T in 8 4 2; do
        timeout -k 10 600 python bench.py --tasks $T --steps ${SHARE_STEPS:-5} --warmup 1 --cpu-sample-steps 0 \
          --adapt-epochs 0 --cfg5-share-tasks 0 > "$O/share_t$T.log" 2>&1
        ok $? "share_t$T"
        echo "tasks=$T $(bench_json "$O/share_t$T.log")" >> "$O/shares.log"
      done ;;
    ab)
      : > "$O/ab.log"
      for round in $(seq 1 "${AB_ROUNDS:-2}"); do
        for v in ${AB_VARIANTS:-base}; do
          extra=""
          case $v in
            arg:*) envs=(); extra=${v#arg:}; extra=${extra//+/ } ;;
            lib:*+opt:*) l=${v#lib:}; envs=(SMAML_LIB=$PKG/${l%%+opt:*} SMAML_OPTIONS=${l#*+opt:}) ;;
            lib:*) envs=(SMAML_LIB=$PKG/${v#lib:}) ;;
            opt:*) envs=(SMAML_OPTIONS=${v#opt:}) ;;
            *) envs=() ;;
          esac
          env "${envs[@]}" timeout -k 10 900 python bench.py ${AB_ARGS:---steps 3 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0} $extra \
            > "$O/ab_tmp.log" 2>&1
          ok $? "ab $v"
          echo "$v $(bench_json "$O/ab_tmp.log")" >> "$O/ab.log"
        done
      done
      python tools/ab_summary.py "$O/ab.log" 2>/dev/null || true ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
