"""Per-kernel SQ instruction mix from a rocprofv3 --pmc pass (`tools/gpu.sh pmc_sq`):
instructions per MFMA and the wait / active fractions of wave time."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"
f = sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True))[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    key = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
cols = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT")
print(f"{'kernel':48s} " + " ".join(f"{c[8:]:>12s}" for c in cols) + "   /mfma  wait/wave  valu/wave")
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    m = c["SQ_INSTS_MFMA"] or 1
    print(f"{k:48s} " + " ".join(f"{c[x] / m:12.2f}" for x in cols) +
          f"   {c['SQ_WAIT_INST_ANY'] / max(c['SQ_WAVE_CYCLES'], 1):9.3f}  {c['SQ_ACTIVE_INST_VALU'] / max(c['SQ_WAVE_CYCLES'], 1):9.3f}")
