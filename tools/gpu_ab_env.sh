#!/bin/bash
# A/B runtime options of one library build on the SO bench: each AB_ENVS entry (';'-separated,
# e.g. "SMAML_OVERLAP=0;SMAML_OVERLAP=1") in its own process, interleaved AB_ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.log
IFS=';' read -ra ENVS <<< "${AB_ENVS:-SMAML_OVERLAP=0;SMAML_OVERLAP=1}"
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for e in "${ENVS[@]}"; do
    env $e timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-sample-steps 0 ${BENCH_ARGS:-} > gpurun_out/ab_tmp.log 2>&1 || exit $?
    echo "${e// /,} $(tail -1 gpurun_out/ab_tmp.log)" >> gpurun_out/ab.log
  done
done
