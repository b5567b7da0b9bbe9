#!/bin/bash
# Config-4 A/B: GPU tests of the adaptation / module-API paths with the default library, then
# tools/bench_adapt.py for each library variant (own process each, interleaved AB_ROUNDS times),
# then a rocprofv3 kernel trace of the default library. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS-tests/test_gpu_adapt.py tests/test_gpu_api.py}" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS-tests/test_gpu_adapt.py tests/test_gpu_api.py} -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_adapt.log 2>&1
  rc=$?
  tail -3 gpurun_out/pytest_adapt.log
  [ $rc -eq 0 ] || exit $rc
fi
: > gpurun_out/ab_adapt.log
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in libsmaml.so ${AB_VARIANTS:-}; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python tools/bench_adapt.py --epochs 2 --warmup 0 \
      --cpu-sample-steps 0 > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/ab_tmp.log | tail -1)" >> gpurun_out/ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/ab_adapt.log"):
    lib, _, js = line.partition(" ")
    r[lib].append(json.loads(js)["later_epoch_ms"] / 960)
for lib, v in r.items():
    print(f"{lib:28s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
rm -rf gpurun_out/prof_adapt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_adapt -o run -- \
  python tools/bench_adapt.py --epochs 2 --warmup 0 --cpu-sample-steps 0 > gpurun_out/prof_adapt.log 2>&1
