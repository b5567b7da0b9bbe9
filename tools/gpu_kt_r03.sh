#!/bin/bash
# Kernel trace + stats of the default bench (rocprofv3), summary printed per kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
BA="${BENCH_ARGS:---steps 2 --warmup 1 --cpu-sample-steps 0 --adapt-epochs 0}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_kt -o run -- python bench.py $BA > gpurun_out/${TAG}_kt.log 2>&1 || exit $?
python - <<PY
import csv, glob
f = glob.glob("gpurun_out/${TAG}_kt/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    n = r["Name"].split("(")[0][:70]
    print(f'{n:72s} calls {int(r["Calls"]):6d} total {float(r["TotalDurationNs"])/1e6:9.1f} ms avg {float(r["AverageNs"])/1e3:9.1f} us {100*float(r["TotalDurationNs"])/tot:5.1f}%')
PY
