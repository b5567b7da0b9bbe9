#!/bin/bash
# Round-4 final at HEAD after the batch-1 launch trims: the whole -m gpu suite, smoke, the default bench
# line, then the config-4 kernel trace (tools/gpu_r04v.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_check_r04b.sh || exit $?
bash tools/gpu_r04v.sh
