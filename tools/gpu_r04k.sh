#!/bin/bash
# Round 4: config-4 A/B of the three-tile forward chunk (LDS copy of the third B image) and of device
# kernel arguments, then the phase probe of the new build. Parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_adapt.py::test_adaptation_n441_matches_oracle" > gpurun_out/r04k_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04k_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r04k_ab_adapt.log
for round in 1 2; do
  for v in "lds3 libsmaml.so" "nolds3 libsmaml_nolds3.so" "devkarg libsmaml.so HIP_FORCE_DEV_KERNARG=1"; do
    set -- $v
    env ${3:-X_=0} SMAML_LIB=weatherforecast_stgcn_maml_amd/$2 timeout -k 10 300 python tools/bench_adapt.py --epochs 2 \
      --warmup 0 --cpu-sample-steps 0 > gpurun_out/r04k_tmp.log 2>&1 || exit $?
    echo "$1 $(grep '^{' gpurun_out/r04k_tmp.log | tail -1)" >> gpurun_out/r04k_ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/r04k_ab_adapt.log"):
    k, _, js = line.partition(" ")
    r[k].append(json.loads(js)["later_epoch_ms"] / 960)
for k, v in r.items():
    print(f"{k:10s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
timeout -k 10 240 python -u tools/kw_probe.py --diag 12 --bdiag 12 > gpurun_out/r04k_probe.log 2>&1 || exit $?
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 240 python -u tools/kw_probe.py --diag 12 --bdiag 12 >> gpurun_out/r04k_probe.log 2>&1 || exit $?
grep -v "amdgpu.ids" gpurun_out/r04k_probe.log
