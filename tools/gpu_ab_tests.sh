#!/bin/bash
# GPU parity tests of the default build, then (only if green) the A/B of library variants on the
# SO bench (tools/gpu_ab.sh). Chain stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh
