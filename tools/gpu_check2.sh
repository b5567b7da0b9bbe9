#!/bin/bash
# GPU tests (incl. adaptation) + a 2-rank gloo rehearsal of bench.py's distributed path on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SMAML_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --tasks 4 --cpu-sample-steps 0 > gpurun_out/bench_2rank.log 2>&1
rc=$?; echo "2-rank rc=$rc"; tail -2 gpurun_out/bench_2rank.log | cut -c1-400
for T in 2 1; do
  timeout -k 10 300 python bench.py --tasks $T --steps 2 --warmup 1 --cpu-sample-steps 0 > gpurun_out/bench_t$T.log 2>&1
  echo "tasks=$T rc=$?"; python tools/ab_summary.py /dev/stdin <<< "t$T $(tail -1 gpurun_out/bench_t$T.log)"
done
