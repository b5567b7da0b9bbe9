#!/bin/bash
# GPU parity tests, then the 15-task bench and the small-grid (per-rank at N=8/N=4) benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for T in ${BENCH_TASKS:-15 4 2}; do
  timeout -k 10 300 python bench.py --tasks $T --steps 2 --warmup 1 --cpu-sample-steps 0 > gpurun_out/bench_t$T.log 2>&1 || exit $?
  python tools/ab_summary.py /dev/stdin <<< "t$T $(tail -1 gpurun_out/bench_t$T.log)"
done
