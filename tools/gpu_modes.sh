#!/bin/bash
# Config-2 bench in the other modes: train-mode dropout 0.2/0.2 (the reference's training setting) and first order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 --dropout 0.2 0.2 > gpurun_out/mode_dropout.log 2>&1 || exit $?
tail -1 gpurun_out/mode_dropout.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 --order 1 > gpurun_out/mode_fo.log 2>&1 || exit $?
tail -1 gpurun_out/mode_fo.log | cut -c1-200
