#!/bin/bash
# Round 4: config-4 A/B of the grouped weight-gradient launch size (wgrad_group_wgs) at batch 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04m_ab_adapt.log
for round in 1 2; do
  for v in 256 128 512 1024; do
    SMAML_OPTIONS=wgrad_group_wgs=$v timeout -k 10 300 python tools/bench_adapt.py --epochs 2 --warmup 0 \
      --cpu-sample-steps 0 > gpurun_out/r04m_tmp.log 2>&1 || exit $?
    echo "wgs=$v $(grep '^{' gpurun_out/r04m_tmp.log | tail -1)" >> gpurun_out/r04m_ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/r04m_ab_adapt.log"):
    k, _, js = line.partition(" ")
    r[k].append(json.loads(js)["later_epoch_ms"] / 960)
for k, v in r.items():
    print(f"{k:10s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
