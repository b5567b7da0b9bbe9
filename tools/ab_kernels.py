"""Per-kernel A/B table from gpurun_out/ab.log (lines: '<lib> <bench json>')."""
import collections
import json
import sys

rows = collections.defaultdict(list)
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    lib, _, js = line.partition(" ")
    try:
        rows[lib].append(json.loads(js))
    except ValueError:
        continue
cats = None
for lib, rs in rows.items():
    cats = cats or list(rs[0].get("kernels", {}).keys())
    ms = sorted(r["ms_per_step"] for r in rs)
    ks = {c: min(r["kernels"][c]["ms_per_step"] for r in rs) for c in cats}
    print(f"{lib:28s} step {ms[0]:8.1f} ms (max {ms[-1]:8.1f}) | " +
          " ".join(f"{c} {ks[c]:.0f}" for c in cats if ks[c] > 1))
