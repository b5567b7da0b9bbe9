#!/bin/bash
# Parity subset with a candidate library (X6_LIB), then a bench A/B against libsmaml.so (the first A/B of the bf16x6 build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
X6=${X6_LIB:-libsmaml.so}
SMAML_LIB=weatherforecast_stgcn_maml_amd/$X6 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -m gpu ${X6_TESTS:-tests/test_gpu_parity.py} > gpurun_out/x6_pytest.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/x6_pytest.log
tail -3 gpurun_out/x6_pytest.log
[ $rc -le 1 ] || exit $rc
: > gpurun_out/ab.log
for round in $(seq 1 ${AB_ROUNDS:-1}); do
  for v in libsmaml.so $X6; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
cat gpurun_out/ab.log
