#!/bin/bash
# Round 4: the small-grid paths at the final HEAD library (adaptation tests, the tile-variant kw / split
# arms, the GPU API module tests), then smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_adapt.py \
  "tests/test_gpu_parity.py::test_second_order_tile_variants_task_groups" tests/test_gpu_compat.py \
  > gpurun_out/r04t_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04t_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -1
