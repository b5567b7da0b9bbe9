"""Per-sample-step kernel breakdown of a rocprofv3 kernel trace of tools/bench_adapt.py
(config 4, batch-1 adaptation): steps are delimited by the Adam kernel (k_adam_l2); averages
over steps of the later epochs (skip the first 1000 steps: first-epoch GCN feature fills).

Usage: python tools/adapt_prof_summary.py gpurun_out/prof_adapt/run_kernel_trace.csv [bench log]
"""
import collections
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    idx = [i for i, x in enumerate(rows) if "k_adam_l2" in x["Kernel_Name"]]
    sel = list(zip(idx[1000:-1], idx[1001:]))
    tot, cnt = collections.Counter(), collections.Counter()
    span = 0
    for a, b in sel:
        span += int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])
        for x in rows[a + 1:b + 1]:
            k = x["Kernel_Name"].split("(")[0].replace("void ", "").replace("smaml::", "")
            tot[k] += int(x["End_Timestamp"]) - int(x["Start_Timestamp"])
            cnt[k] += 1
    n = len(sel)
    print(f"# config-4 sample-step kernel breakdown ({n} later-epoch steps of {sys.argv[1]})\n")
    if len(sys.argv) > 2:
        for line in open(sys.argv[2]):
            if line.startswith("{"):
                d = json.loads(line)
                print(f"bench (under the profiler): {d['ms_per_sample_step']:.3f} ms per sample-step over "
                      f"{d['epochs']} epochs, later epochs {d['later_epoch_ms'] / d['config']['train_samples']:.3f} ms\n")
    print("| kernel | us / step | launches / step |\n|---|---|---|")
    for k, v in tot.most_common():
        print(f"| `{k}` | {v / n / 1000:.1f} | {cnt[k] / n:.1f} |")
    print(f"| **sum of kernel time** | **{sum(tot.values()) / n / 1000:.1f}** | {sum(cnt.values()) / n:.0f} |")
    print(f"\nstep span (Adam end to Adam end): {span / n / 1000:.1f} us")


if __name__ == "__main__":
    main()
