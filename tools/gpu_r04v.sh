#!/bin/bash
# Round 4: config-4 kernel trace at HEAD (tools/bench_adapt.py, 2 epochs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/r04v_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04v_prof -o run -- \
  python tools/bench_adapt.py --epochs 2 --warmup 0 --cpu-sample-steps 0 > gpurun_out/r04v_prof.log 2>&1
echo "prof rc=$?"
