#!/bin/bash
# Round 4: batch-1 forward with layer 0's input projection hoisted out of the wavefront (one GEMM for all
# steps): parity (adaptation, tile variants, module API), then config-4 A/B against the previous build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_adapt.py \
  "tests/test_gpu_parity.py::test_second_order_tile_variants_task_groups" tests/test_gpu_compat.py \
  > gpurun_out/r04u_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04u_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r04u_ab_adapt.log
for round in 1 2; do
  for v in libsmaml.so libsmaml_prev.so; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python tools/bench_adapt.py --epochs 2 --warmup 0 \
      --cpu-sample-steps 0 > gpurun_out/r04u_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/r04u_tmp.log | tail -1)" >> gpurun_out/r04u_ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/r04u_ab_adapt.log"):
    k, _, js = line.partition(" ")
    r[k].append(json.loads(js)["later_epoch_ms"] / 960)
for k, v in r.items():
    print(f"{k:20s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
