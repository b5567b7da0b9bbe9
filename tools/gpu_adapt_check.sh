#!/bin/bash
# Config-4 (batch-1 adaptation) check: GPU tests of the adaptation / module-API paths, then the
# adaptation bench under rocprofv3 kernel tracing. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_adapt.py tests/test_gpu_api.py} -x -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_adapt.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_adapt.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_adapt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_adapt -o run -- \
  python tools/bench_adapt.py --epochs ${EPOCHS:-3} --warmup 0 --cpu-sample-steps 0 > gpurun_out/prof_adapt.log 2>&1
rc=$?
grep '^{' gpurun_out/prof_adapt.log | tail -1
exit $rc
