#!/bin/bash
# rocprofv3 kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) on the
# hot kernels. Writes under gpurun_out/prof_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BA="${BENCH_ARGS:---steps 2 --warmup 1 --cpu-sample-steps 0}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt -o run -- python bench.py $BA > gpurun_out/prof_kt.log 2>&1 || exit $?
echo "kernel-trace ok"
RX="${PMC_REGEX:-k_lstm_fwd|k_lstm_bwd|k_wgrad|k_gcn_layer|k_gemm_nn}"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-include-regex "$RX" -f csv -d gpurun_out/prof_pmc_$C -o run -- python bench.py --steps 1 --warmup 0 --cpu-sample-steps 0 --no-timing > gpurun_out/prof_pmc_$C.log 2>&1 || exit $?
  echo "pmc $C ok"
done
