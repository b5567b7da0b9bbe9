#!/bin/bash
# Diagnostic: the STGCN autograd test alone in a fresh process with serialized, checked kernel launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_api.py::test_stgcn_autograd_matches_oracle" "tests/test_gpu_parity.py::test_gcnconv_dropin_matches_oracle" > gpurun_out/diag_stgcn.log 2>&1
rc=$?
grep -E "PASSED|FAILED|rror|smaml" gpurun_out/diag_stgcn.log | head -30
exit $rc
