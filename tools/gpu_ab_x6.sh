#!/bin/bash
# Accuracy test (f32 and x6 builds) + bench A/B over library variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/acc.log
for v in ${ACC_LIBS:-}; do
  SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread \
    -m gpu tests/test_gpu_accuracy.py >> gpurun_out/acc.log 2>&1
  rc=$?; echo "$v accuracy exit $rc" >> gpurun_out/acc.log
  [ $rc -le 1 ] || exit $rc
done
grep -E "worst|exit|passed|failed" gpurun_out/acc.log
: > gpurun_out/ab.log
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in ${AB_VARIANTS}; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
python tools/ab_summary.py gpurun_out/ab.log 2>/dev/null || true
