#!/bin/bash
# Round 4 end: the per-rank shares of the 15-task meta-batch at N = 2 / 4 / 8 (8 / 4 / 2 tasks: rank 0's
# round-robin share) and the full 15, timed on one GPU -- the single-GPU basis of the scaling prediction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04_shares.log
for t in 15 8 4 2; do
  timeout -k 10 300 python bench.py --tasks $t --adapt-epochs 0 --cfg5-share-tasks 0 --cpu-sample-steps 0 \
    > gpurun_out/r04_shares_tmp.log 2>&1 || exit $?
  echo "tasks=$t $(grep '^{' gpurun_out/r04_shares_tmp.log | tail -1)" >> gpurun_out/r04_shares.log
done
python - <<'PY'
import json
r = {}
for line in open("gpurun_out/r04_shares.log"):
    k, _, js = line.partition(" ")
    r[int(k.split("=")[1])] = json.loads(js)["ms_per_step"]
for t in (15, 8, 4, 2):
    print(f"{t:2d} tasks: {r[t]:8.1f} ms per meta-step; 15-task time / this = {r[15] / r[t]:.2f}x")
PY
