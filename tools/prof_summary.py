"""Summarise a rocprofv3 run (kernel stats + FETCH_SIZE/WRITE_SIZE PMC passes) into markdown,
and optionally write the per-launch HBM traffic of each bench timing category as JSON
(``bench.py`` reads it into ``roofline.traffic`` when the per-rank workload matches: the file holds one
entry per profiled rank workload, e.g. 15 tasks for N=1 and the 8/4/2-task rank shares for N=2/4/8).

FETCH_SIZE on gfx950 reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md §HBM, 16 B/lane loads as all our operand loads are): the corrected
figure doubles it. WRITE_SIZE is exact for 16-B streaming stores; our epilogue stores are
4-B scattered stores (uncalibrated width), so the write column is indicative. Units: KB.

Usage: prof_summary.py RUN_DIR TITLE [TRAFFIC_JSON PROFILE_MD]
(the workload string is taken from the profiled bench's JSON line in RUN_DIR/prof_kt.log)
"""
import collections
import csv
import json
import os
import re
import sys

# bench.py timing categories (api.cpp TIMED(...)) -> the kernels each category launches
CATEGORIES = {
    "gcn_layer": r"k_gcn_layer|k_gcn_mlp|k_gcn_expand|k_gcn_compact",
    "lstm_fwd_step": r"k_lstm_fwd_step",
    "lstm_fwd_dual": r"k_lstm_fwd_dual",
    "lstm_bwd_step": r"k_lstm_bwd_step",
    "lstm_bwd_dual": r"k_lstm_bwd_dual",
    "wgrad": r"k_wgrad$|k_wgrad\b(?!_)",
    "wgrad_reduce": r"k_wgrad_reduce",
    "head_dh": r"k_gemm_nn",
    "head_loss": r"k_head_(loss|dual)",
    "xg_proj": r"k_xg_dedup|k_gemm_nt",
    "dg_rowsum": r"k_dg_rowsum",
}


def short(name):
    return name.split("(")[0].replace("smaml::", "").replace("void ", "")


def kstats(d):
    p = os.path.join(d, "prof_kt", "run_kernel_stats.csv")
    out = []
    for r in csv.DictReader(open(p)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                    float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def pmc(d, c):
    """kernel full name -> list of per-dispatch counter values (KB)."""
    p = os.path.join(d, f"prof_pmc_{c}", "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return agg


def bench_line(d):
    for line in reversed(open(os.path.join(d, "prof_kt.log")).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main(d, title, traffic_out=None, profile_md=None):
    ks = kstats(d)
    print(f"# {title}\n")
    print("rocprofv3 --kernel-trace --stats of `bench.py` (config 2); times summed over the profiled run.\n")
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---|---|---|---|")
    for n, c, t, a, p in ks:
        if p >= 0.01:
            print(f"| {short(n)} | {c} | {t:.1f} | {a:.1f} | {p:.2f} |")

    print("\nPer bench timing category (the same kernels `bench.py`'s HIP events bracket):\n")
    print("| category | kernels | calls | total ms | avg us per launch |")
    print("|---|---|---|---|---|")
    cat_stats = {}
    for cat, rx in CATEGORIES.items():
        sel = [(n, c, t) for n, c, t, _, _ in ks if re.search(rx, n)]
        if not sel:
            continue
        calls = sum(c for _, c, _ in sel)
        tot = sum(t for _, _, t in sel)
        cat_stats[cat] = (calls, tot)
        print(f"| {cat} | {', '.join(sorted({short(n) for n, _, _ in sel}))} | {calls} | {tot:.1f} | "
              f"{tot * 1e3 / calls:.1f} |")

    f, w = pmc(d, "FETCH_SIZE"), pmc(d, "WRITE_SIZE")
    if not f:
        return
    print("\nPMC (separate `--pmc` passes, per-dispatch average; FETCH x2 = gfx950 correction):\n")
    print("| kernel | dispatches | FETCH_SIZE MB | FETCH x2 MB | WRITE_SIZE MB |")
    print("|---|---|---|---|---|")
    for k in f:
        fa = sum(f[k]) / len(f[k])
        wa = sum(w.get(k, [0])) / max(len(w.get(k, [0])), 1)
        print(f"| {short(k)} | {len(f[k])} | {fa / 1024:.1f} | {2 * fa / 1024:.1f} | {wa / 1024:.1f} |")
    traffic = {}
    print("\nHBM traffic per category launch (FETCH x2 + WRITE, dispatch-weighted):\n")
    print("| category | dispatches | read MB | write MB | total MB |")
    print("|---|---|---|---|---|")
    for cat, rx in CATEGORIES.items():
        fr = [v for k, vs in f.items() if re.search(rx, k) for v in vs]
        wr = [v for k, vs in w.items() if re.search(rx, k) for v in vs]
        if not fr:
            continue
        rd = 2 * sum(fr) / len(fr) * 1024
        wt = (sum(wr) / len(wr) * 1024) if wr else 0.0
        per = 1.0  # one kernel per timing category
        traffic[cat] = {"read_bytes": rd * per, "write_bytes": wt * per, "bytes_per_launch": (rd + wt) * per}
        print(f"| {cat} | {len(fr)} | {rd * per / 1e6:.1f} | {wt * per / 1e6:.1f} | {(rd + wt) * per / 1e6:.1f} |")
    if traffic_out:
        # merge into {"profiles": {rank workload key (bench.py rank_workload): {...}}}
        b = bench_line(d)
        key = (b.get("rank_workload") or b["config"]["workload"]) if b else None
        doc = {"unit": "bytes", "profiles": {}}
        if os.path.exists(traffic_out):
            try:
                old = json.load(open(traffic_out))
                doc["profiles"] = old.get("profiles", {})
            except ValueError:
                pass
        doc["profiles"][key] = {"profile": profile_md, "categories": traffic}
        json.dump(doc, open(traffic_out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profile",
         sys.argv[3] if len(sys.argv) > 3 else None, sys.argv[4] if len(sys.argv) > 4 else None)
