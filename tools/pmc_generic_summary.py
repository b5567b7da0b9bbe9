"""Per-kernel sums of every counter in rocprofv3 --pmc output directories, plus derived ratios.

usage: pmc_generic_summary.py DIR [DIR ...]   (each DIR holds a run's counter_collection.csv)
Derived (when the counters are present): mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4)
(SQ_BUSY_CYCLES counts per SE... printed raw as well), wait fractions per wave-cycle."""
import collections
import csv
import glob
import sys

for root in sys.argv[1:]:
    files = sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True))
    if not files:
        print(root, "no csv")
        continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(files[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = name.replace("smaml::", "")[:70]
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[key][r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    print(f"== {root}")
    for k, c in sorted(acc.items(), key=lambda kv: -sum(e - s for s, e in disp[kv[0]].values())):
        wall = sum(e - s for s, e in disp[k].values()) * 1e-6
        line = f"{k:70s} n={len(disp[k]):4d} ms={wall:8.1f}"
        wc = c.get("SQ_WAVE_CYCLES")
        for n, v in sorted(c.items()):
            line += f" {n}={v:.4g}"
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    line += f" {n}/wave_cyc={c[n] / wc:.3f}"
        if "SQ_INSTS_MFMA" in c and "SQ_INSTS_VALU" in c:
            line += f" valu/mfma={c['SQ_INSTS_VALU'] / c['SQ_INSTS_MFMA']:.2f}"
        print(line)
