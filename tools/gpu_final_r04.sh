#!/bin/bash
# Round-4 final: full -m gpu suite, smoke, default bench line, then the 15-task FETCH/WRITE passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_check_r04b.sh || exit $?
TASKS=15 bash tools/gpu_prof_r04.sh || exit $?
