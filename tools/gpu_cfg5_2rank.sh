#!/bin/bash
# Config-5 rank share (8 tasks, N=1024, Hc=512, K=10) and a 2-rank self-launched bench over gloo on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config 5 --tasks 8 --steps 1 --warmup 1 > gpurun_out/cfg5_share8.log 2>&1 || exit $?
tail -1 gpurun_out/cfg5_share8.log | cut -c1-300
SMAML_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 1 --cpu-sample-steps 0 > gpurun_out/bench_2rank_gloo.log 2>&1 || exit $?
tail -1 gpurun_out/bench_2rank_gloo.log | cut -c1-400
