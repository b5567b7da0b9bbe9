#!/bin/bash
# Config-4 adaptation bench (default lib and the f32-MFMA build) and per-rank share benches
# (tasks 8/4/2 = the slowest rank at 2/4/8 GPUs) for the scaling prediction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in libsmaml.so libsmaml_f32.so; do
  SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python tools/bench_adapt.py --epochs 2 --warmup 0 \
    --cpu-sample-steps 0 > gpurun_out/adapt_$v.log 2>&1 || exit $?
  echo "adapt $v $(tail -1 gpurun_out/adapt_$v.log | cut -c1-300)"
done
for n in 8 4 2; do
  timeout -k 10 300 python bench.py --tasks $n --steps 3 --warmup 1 --cpu-sample-steps 0 > gpurun_out/share_$n.log 2>&1 || exit $?
  echo "tasks $n $(tail -1 gpurun_out/share_$n.log | cut -c1-200)"
done
