#!/bin/bash
# Round-3 scaling evidence on one GPU: the slowest rank's share at 2/4/8 GPUs (8/4/2 tasks of the
# 15-task meta-batch), config 5's rank share at 8 GPUs, and the self-launched 2-rank bench over gloo.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 8 4 2; do
  timeout -k 10 300 python bench.py --tasks $n --steps 3 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 > gpurun_out/share_$n.log 2>&1 || exit $?
  echo "tasks $n $(tail -1 gpurun_out/share_$n.log | cut -c1-160)"
done
timeout -k 10 400 python bench.py --config 5 --tasks 8 --steps 1 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 > gpurun_out/cfg5_share8.log 2>&1 || exit $?
echo "cfg5 $(tail -1 gpurun_out/cfg5_share8.log | cut -c1-200)"
SMAML_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 > gpurun_out/bench_2rank_gloo.log 2>&1 || exit $?
echo "2rank $(tail -1 gpurun_out/bench_2rank_gloo.log | cut -c1-300)"
