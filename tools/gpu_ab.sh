#!/bin/bash
# A/B the library variants on the SO bench (each in its own process, interleaved twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -x ./tools/gemm_micro ]; then timeout -k 10 300 ./tools/gemm_micro > gpurun_out/micro.log 2>&1 || exit $?; fi
: > gpurun_out/ab.log
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in libsmaml.so ${AB_VARIANTS:-libsmaml_bk16.so libsmaml_gate16.so}; do
    SMAML_LIB=weatherforecast_stgcn_maml_amd/$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "$v $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
