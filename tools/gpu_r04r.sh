#!/bin/bash
# Round 4: careful A/B of the tangent BPTT's pair-segment tile order (bwdd_remap) on the headline bench,
# three interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/ab_run.py gpurun_out/r04r_ab.log 3 base=libsmaml.so remap=libsmaml.so:SMAML_OPTIONS=bwdd_remap=1
