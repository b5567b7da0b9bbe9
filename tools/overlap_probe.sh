#!/bin/bash
# Does running two independent task chains concurrently fill the GEMM/epilogue phase gaps?
# One bench process with one 5-task group alone, then two such processes at once on the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
BA="--tasks 5 --steps ${STEPS:-6} --warmup 1 --cpu-sample-steps 0 --no-timing"
timeout -k 10 300 python bench.py $BA > gpurun_out/ov_alone.log 2>&1 || exit $?
echo "alone: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_alone.log)"
t0=$(date +%s.%N)
timeout -k 10 400 python bench.py $BA > gpurun_out/ov_a.log 2>&1 &
pa=$!
timeout -k 10 400 python bench.py $BA > gpurun_out/ov_b.log 2>&1 &
pb=$!
wait $pa; ra=$?
wait $pb; rb=$?
t1=$(date +%s.%N)
echo "pair: a $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_a.log) rc=$ra | b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ov_b.log) rc=$rb | wall $(echo "$t1 - $t0" | bc) s"
tail -2 gpurun_out/ov_a.log gpurun_out/ov_b.log | grep -v '^{' | head -6
