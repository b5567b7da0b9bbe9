#!/bin/bash
# Round 4: the one-launch small-grid LSTM steps (kernels_small.hip, option small_kw). Parity of the
# N=441 adaptation against the oracle on both small-grid paths, then config 4 timed with small_kw 0 / 1
# (tools/bench_adapt.py, 2 epochs, interleaved; 2 = with BPTT images), then a kernel trace of small_kw=2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_adapt.py::test_adaptation_n441_matches_oracle" "tests/test_gpu_adapt.py::test_adaptation_fused_update_bitwise" \
  > gpurun_out/r04h_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04h_pytest.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r04h_ab_adapt.log
for round in 1 2; do
  for kw in 0 1 2 "2,grid_barrier=0"; do
    SMAML_OPTIONS=small_kw=$kw timeout -k 10 300 python tools/bench_adapt.py --epochs 2 --warmup 0 \
      --cpu-sample-steps 0 > gpurun_out/r04h_tmp.log 2>&1 || exit $?
    echo "small_kw=$kw $(grep '^{' gpurun_out/r04h_tmp.log | tail -1)" >> gpurun_out/r04h_ab_adapt.log
  done
done
python - <<'PY'
import json, collections
r = collections.defaultdict(list)
for line in open("gpurun_out/r04h_ab_adapt.log"):
    k, _, js = line.partition(" ")
    r[k].append(json.loads(js)["later_epoch_ms"] / 960)
for k, v in r.items():
    print(f"{k:12s} later-epoch ms/sample-step: " + " ".join(f"{x:.3f}" for x in v))
PY
rm -rf gpurun_out/r04h_prof
SMAML_OPTIONS=small_kw=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r04h_prof -o run -- \
  python tools/bench_adapt.py --epochs 2 --warmup 0 --cpu-sample-steps 0 > gpurun_out/r04h_prof.log 2>&1
echo "prof rc=$?"
