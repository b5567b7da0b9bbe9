"""Per-kernel comparison of bench lines: python tools/bench_cmp.py LOG [LOG ...] (each file's last JSON line)."""
import json
import sys

for f in sys.argv[1:]:
    j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    ex = j.get("executed_tflop")
    print(f"{f}: {j['ms_per_step']:.1f} ms/meta-step" + (f", executed {ex:.1f} TFLOP" if ex else "") +
          (f", roofline {j['roofline']['kernel']} {j['roofline']['frac']:.3f}" if "roofline" in j else ""))
    for k, v in j.get("kernels", {}).items():
        print(f"    {k:14s} {v['ms_per_step']:8.1f} ms {v['tflops']:7.1f} TF/s {v['launches_per_step']:7.0f} launches")
    c5 = j.get("config5_rank_share")
    if c5:
        print(f"  config-5 share {c5['value']:.1f} ms: " +
              " ".join(f"{k} {v['ms_per_step']:.0f}" for k, v in c5.get("kernels", {}).items()))
