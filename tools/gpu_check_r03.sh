#!/bin/bash
# Round-3 GPU check: the -m gpu suite (or the test ids in $TESTS), smoke, then the default bench.
# Each GPU step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/} \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${SMOKE-1}" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ -n "${BENCH-1}" ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
fi
if [ -n "${AB_VARIANTS:-}" ]; then
  : > gpurun_out/${TAG}_ab.log
  for round in $(seq 1 ${AB_ROUNDS:-2}); do
    for v in libsmaml.so ${AB_VARIANTS}; do
      SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0 --cfg5-share-tasks 0 ${AB_BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
      echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/${TAG}_ab.log
    done
  done
  python tools/ab_summary.py gpurun_out/${TAG}_ab.log
fi
