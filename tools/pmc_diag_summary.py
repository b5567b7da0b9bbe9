"""Per-kernel summary of tools/gpu_pmc_diag.sh's passes (gpurun_out/pmc_diag_*/**/*counter_collection.csv):
counter totals per kernel symbol (dispatch-summed) and derived ratios."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(f"{root}/pmc_diag_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        k = k.replace("smaml::", "")[:70]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(k)
    for name in sorted(c):
        print(f"   {name:32s} {c[name]:.4g}")
    if "SQ_WAIT_ANY" in c:
        print(f"   -> wait_any/wave_cycles {c['SQ_WAIT_ANY'] / wc:.3f}  wait_inst/wave {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}  "
              f"active/wave {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f}")
    if "TCC_HIT_sum" in c:
        h, m = c["TCC_HIT_sum"], c.get("TCC_MISS_sum", 0)
        print(f"   -> L2 hit rate {h / max(h + m, 1):.3f}")
    if "TCP_TCC_READ_REQ_LATENCY_sum" in c:
        print(f"   -> mean L2 read latency (cycles) {c['TCP_TCC_READ_REQ_LATENCY_sum'] / max(c.get('TCP_TCC_READ_REQ_sum', 1), 1):.1f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        print(f"   -> mfma busy (per CU-cycle) {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 256 * 4) :.3f} (approx)")
