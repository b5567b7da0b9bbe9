#!/bin/bash
# Parity (gpu parity + accuracy tests) on a candidate library, then a bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SMAML_LIB=weatherforecast_stgcn_maml_amd/$CAND timeout -k 10 600 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread \
  -m gpu ${TESTS:-tests/test_gpu_accuracy.py tests/test_gpu_parity.py} > gpurun_out/cand_pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/cand_pytest.log
grep -E "worst|passed|failed|Error|error" gpurun_out/cand_pytest.log | head -20
[ $rc -le 1 ] || exit $rc
: > gpurun_out/ab.log
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in ${AB_VARIANTS}; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
python tools/ab_summary.py gpurun_out/ab.log
