#!/bin/bash
# Round 4 check at HEAD: the whole -m gpu suite, smoke, the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r04i_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04i_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04i_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04i_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04i_bench.log 2> gpurun_out/r04i_bench.err
rc=$?
tail -c 1500 gpurun_out/r04i_bench.log
exit $rc
