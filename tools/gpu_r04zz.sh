#!/bin/bash
# Round 4: consecutive windows on the per-layer GCN path (Hc != 256, e.g. config 5) -- the whole -m gpu
# suite, then the config-5 rank share with gcn_dedup off / on (two interleaved rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04zz_pytest.log 2>&1 || { tail -30 gpurun_out/r04zz_pytest.log; exit 1; }
tail -3 gpurun_out/r04zz_pytest.log
: > gpurun_out/r04zz_ab.log
for round in 1 2; do
  for v in "gcn_dedup=0" "gcn_dedup=1"; do
    SMAML_OPTIONS=$v timeout -k 10 300 python bench.py --steps 1 --warmup 1 --adapt-epochs 0 --cpu-sample-steps 0 \
      > gpurun_out/r04zz_tmp.log 2>&1 || exit $?
    echo "$v $(grep '^{' gpurun_out/r04zz_tmp.log | tail -1)" >> gpurun_out/r04zz_ab.log
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/r04zz_ab.log"):
    k, _, js = line.partition(" ")
    j = json.loads(js)
    c5 = j["config5_rank_share"]
    print(f"{k:14s} config 2 {j['ms_per_step']:.1f} ms  config-5 share {c5['value']:.1f} ms  qmse {c5['query_mse']!r}")
PY
