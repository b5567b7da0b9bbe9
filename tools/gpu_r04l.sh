#!/bin/bash
# Round 4: the 2-rank rehearsal on one GPU (gloo) at the default 15-task meta-batch and at 4 tasks: the
# N>1 line with collective timings and roofline.traffic from the per-rank workload's profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for T in 15 4; do
  SMAML_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --tasks $T --steps 2 --warmup 1 --adapt-epochs 0 \
    --cfg5-share-tasks 0 --cpu-sample-steps 0 > gpurun_out/r04l_gloo_t$T.log 2> gpurun_out/r04l_gloo_t$T.err || { tail -5 gpurun_out/r04l_gloo_t$T.err; exit 1; }
  python - $T <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/r04l_gloo_t{sys.argv[1]}.log") if x.startswith("{")][-1]
j = json.loads(l)
print(sys.argv[1], "tasks: ms_per_step", round(j["ms_per_step"], 1), "collective", j.get("collective"),
      "traffic", j["roofline"].get("traffic"), j["roofline"].get("traffic_source"))
PY
done
