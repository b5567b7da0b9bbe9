#!/bin/bash
# Round 4: batch-1 launch trims -- the adaptation cache filled up front in batched GCN passes
# (api.cpp ad_cache_fill), the head's dh_T inside the head weight-gradient launch, the step loss
# summed by the Adam launch -- and the C-ABI RCCL check. GPU tests, then config-4 first/later-epoch
# times: HEAD's library (libsmaml_prev.so) vs this one with the per-step fill (adapt_gcn_batch=0) vs default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_adapt.py tests/test_gpu_distributed.py tests/test_gpu_api.py > gpurun_out/r04x_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r04x_pytest.log; exit 1; }
tail -3 gpurun_out/r04x_pytest.log
: > gpurun_out/r04x_ab_adapt.log
for round in 1 2; do
  for v in "libsmaml_prev.so:" "libsmaml.so:adapt_gcn_batch=0" "libsmaml.so:"; do
    SMAML_OPTIONS=${v#*:} SMAML_LIB=weatherforecast_stgcn_maml_amd/${v%%:*} timeout -k 10 300 python tools/bench_adapt.py \
      --epochs 2 --warmup 0 --cpu-sample-steps 0 > gpurun_out/r04x_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/r04x_tmp.log | tail -1)" >> gpurun_out/r04x_ab_adapt.log
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r04x_ab_adapt.log"):
    k, _, js = line.partition(" ")
    j = json.loads(js)
    print(f"{k:32s} first epoch {j['first_epoch_ms']:.1f} ms, later epoch {j['later_epoch_ms']:.1f} ms "
          f"({j['later_epoch_ms'] / 960:.4f} ms/sample-step)")
PY
