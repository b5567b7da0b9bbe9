#!/bin/bash
# A/B of run-time knobs on the SO bench: AB_SPECS="label:VAR=value,VAR2=value label2:..." (one
# process per spec, interleaved AB_ROUNDS times), after the parity tests in TESTS (if set).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_ab.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_ab.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/ab.log
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for spec in ${AB_SPECS}; do
    label=${spec%%:*}
    envs=${spec#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 \
      ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$label $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
python tools/ab_kernels.py gpurun_out/ab.log
