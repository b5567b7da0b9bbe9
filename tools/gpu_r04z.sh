#!/bin/bash
# Round 4: the fused GCN rows of consecutive windows once per distinct stream row (k_gcn_mlp dedup,
# option gcn_dedup) -- the whole -m gpu suite and smoke, then the config-2 bench with the option off / on
# (two interleaved rounds, adaptation and config-5 share skipped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04z_pytest.log 2>&1 || { tail -30 gpurun_out/r04z_pytest.log; exit 1; }
tail -3 gpurun_out/r04z_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04z_smoke.log
: > gpurun_out/r04z_ab.log
for round in 1 2; do
  for v in "gcn_dedup=0" "gcn_dedup=1"; do
    SMAML_OPTIONS=$v timeout -k 10 300 python bench.py --adapt-epochs 0 --cfg5-share-tasks 0 --cpu-sample-steps 0 \
      > gpurun_out/r04z_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/r04z_tmp.log | tail -1)" >> gpurun_out/r04z_ab.log
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r04z_ab.log"):
    k, _, js = line.partition(" ")
    j = json.loads(js)
    print(f"{k:14s} {j['ms_per_step']:.1f} ms/meta-step  gcn {j['kernels']['gcn_layer']['ms_per_step']:.1f} ms  "
          f"qmse {j['query_mse']!r}")
PY
