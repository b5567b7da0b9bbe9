#!/bin/bash
# Round-4 final at HEAD (full -m gpu suite, smoke, bench, 15-task FETCH/WRITE passes), then the A/B of the
# grid-row problem index for the small-grid kernels (libsmaml_py.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_final_r04.sh || exit $?
bash tools/gpu_r04s.sh
