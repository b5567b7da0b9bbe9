"""Per-kernel MFMA utilisation / effective clock from a rocprofv3 --pmc MFMA-busy pass (the round-1..3 sessions; `tools/gpu.sh pmc_sq` now).

busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs); clock = kernel cycles / wall time."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_mfma"
f = sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True))[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    key = name[:60]
    d = r["Dispatch_Id"]
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[key][d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
print(f"{'kernel':60s} {'n':>4s} {'ms':>8s} {'GHz':>5s} {'mfma_busy':>9s} {'busy/mfma':>9s}")
for k, c in sorted(acc.items(), key=lambda kv: -sum(e - s for s, e in disp[kv[0]].values())):
    wall = sum(e - s for s, e in disp[k].values()) * 1e-9
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    ghz = cyc / wall / 1e9 if wall else 0
    busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc) if cyc else 0
    per = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"] if c["SQ_INSTS_MFMA"] else 0
    print(f"{k:60s} {len(disp[k]):4d} {wall * 1e3:8.1f} {ghz:5.2f} {busy:9.3f} {per:9.1f}")
