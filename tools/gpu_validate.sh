#!/bin/bash
# Round validation on one box: full -m gpu suite, smoke, default bench, rocprofv3 kernel trace +
# FETCH/WRITE passes, MFMA-busy pass. Every GPU step under its own timeout; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/val_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/val_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/val_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/val_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/val_bench.log 2>&1 || exit $?
tail -1 gpurun_out/val_bench.log | cut -c1-400
bash tools/gpu_profile.sh || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_" -f csv -d gpurun_out/pmc_mfma -o run -- python bench.py --steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing > gpurun_out/pmc_mfma.log 2>&1 || exit $?
python tools/pmc_mfma_summary.py gpurun_out/pmc_mfma > gpurun_out/pmc_mfma.txt 2>&1
head -8 gpurun_out/pmc_mfma.txt
