#!/bin/bash
# Round 4: config-4 A/B of the forward's weight operand at batch 1 -- pre-split gate images (k_split_gate
# every step) vs f32 weights split in registers (gate_img=0) -- and of the hoisted projection's tiles
# (libsmaml_ntbig.so: 256 x 128).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04w_ab_adapt.log
for round in 1 2; do
  for v in "libsmaml.so:" "libsmaml.so:gate_img=0" "libsmaml_ntbig.so:"; do
    SMAML_OPTIONS=${v#*:} SMAML_LIB=weatherforecast_stgcn_maml_amd/${v%%:*} timeout -k 10 300 python tools/bench_adapt.py \
      --epochs 2 --warmup 0 --cpu-sample-steps 0 > gpurun_out/r04w_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/r04w_tmp.log | tail -1)" >> gpurun_out/r04w_ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/r04w_ab_adapt.log"):
    k, _, js = line.partition(" ")
    r[k].append(json.loads(js)["later_epoch_ms"] / 960)
for k, v in r.items():
    print(f"{k:20s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
