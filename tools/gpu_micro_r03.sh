#!/bin/bash
# Round-3 micro-benchmarks (each under its own time limit), then the regular check script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/micro.log
for m in ${MICROS:-}; do
  echo "== $m" >> gpurun_out/micro.log
  timeout -k 10 120 ./tools/$m >> gpurun_out/micro.log 2>&1 || exit $?
done
cat gpurun_out/micro.log
[ -n "${CHECK:-1}" ] && exec_rc=0 && bash tools/gpu_check_r03.sh
