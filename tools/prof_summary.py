"""Summarise a rocprofv3 run (kernel stats + FETCH_SIZE/WRITE_SIZE PMC passes) into markdown.

FETCH_SIZE on gfx950 reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md §HBM): the 'corrected' column doubles it. Units are KB.
"""
import collections
import csv
import os
import sys


def kstats(d):
    p = os.path.join(d, "prof_kt", "run_kernel_stats.csv")
    out = []
    for r in csv.DictReader(open(p)):
        out.append((r["Name"].split("(")[0].replace("smaml::", ""), int(r["Calls"]),
                    float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def pmc(d, c):
    p = os.path.join(d, f"prof_pmc_{c}", "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"].split("(")[0].replace("smaml::", "")].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(d, title):
    print(f"# {title}\n")
    print("rocprofv3 --kernel-trace --stats (bench.py, config 2); times summed over the profiled run.\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for n, c, t, a, p in kstats(d):
        if p >= 0.01:
            print(f"| {n} | {c} | {t:.1f} | {a:.1f} | {p:.2f} |")
    f, w = pmc(d, "FETCH_SIZE"), pmc(d, "WRITE_SIZE")
    if f:
        print("\nPMC (separate passes, per dispatch average, MB = KB/1024):\n")
        print("| kernel | FETCH_SIZE MB | x2 corrected MB | WRITE_SIZE MB |")
        print("|---|---|---|---|")
        for k in f:
            print(f"| {k} | {f[k] / 1024:.1f} | {2 * f[k] / 1024:.1f} | {w.get(k, 0) / 1024:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profile")
