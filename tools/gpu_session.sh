#!/bin/bash
# One GPU-box session (chain stops at the first crash-like exit):
#   [micro]  tools/gate_micro (tile / epilogue variants on the config-2 LSTM shapes)
#   [tests]  pytest -m gpu, smoke()
#   [bench]  default bench line (config 2, second order) -> gpurun_out/bench.json
#   [prof]   rocprofv3 --kernel-trace --stats of the bench + FETCH_SIZE / WRITE_SIZE passes
# STEPS selects a subset, e.g. STEPS="tests bench".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-micro tests bench prof}"
ok() { # rc name
  local rc=$1
  echo "$2 rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
}
for s in $STEPS; do
  case $s in
    micro)
      timeout -k 10 300 ./tools/gate_micro > gpurun_out/gate_micro.log 2>&1; ok $? micro ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; ok $? pytest
      tail -3 gpurun_out/pytest_gpu.log
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $? smoke
      tail -2 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; ok $? bench
      tail -1 gpurun_out/bench.log > gpurun_out/bench.json ;;
    prof)
      PA="--steps 2 --warmup 1 --cpu-sample-steps 0"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt -o run -- \
        python bench.py $PA > gpurun_out/prof_kt.log 2>&1; ok $? prof_kt
      RX="${PMC_REGEX:-k_lstm_fwd|k_lstm_bwd|k_wgrad|k_gcn_layer|k_gemm_nn}"
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d gpurun_out/prof_pmc_$C -o run -- \
          python bench.py --steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing > gpurun_out/prof_pmc_$C.log 2>&1
        ok $? pmc_$C
      done ;;
  esac
done
