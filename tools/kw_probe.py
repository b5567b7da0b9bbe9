"""Phase timeline of the small-grid LSTM kernels (kernels_small.hip) from a probe build.

Build (here, CPU): python tools/kw_probe.py --build      -> weatherforecast_stgcn_maml_amd/libsmaml_kwprobe.so
Run (GPU box):     python tools/kw_probe.py [--diag 12] [--bdiag 12]

Runs BASELINE config-4 shaped batch-1 adaptation steps (N=441, Hc=256, LSTM 4x128) through the probe
library, with the probe armed on one forward diagonal and then one BPTT diagonal; each workgroup's
wave 0 records wall_clock64 at kernel entry, K-loop loads issued, K loop done, partial tiles
in LDS, epilogue issued. Prints, relative to the earliest entry of the launch, the median / max of each
phase and the spread of entries and of ends.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "weatherforecast_stgcn_maml_amd", "libsmaml_kwprobe.so")


def report(name, ts, tick_ns):
    ts = ts[(ts[:, 0] > 0) & (ts[:, 4] > 0)].astype(np.float64)
    if len(ts) == 0:
        print(f"{name}: no samples")
        return
    t0 = ts[:, 0].min()
    rel = (ts - t0) * tick_ns / 1000.0  # us
    ph = np.diff(rel, axis=1)
    names = ["prologue+issue", "K loop", "LDS write+barrier", "epilogue"]
    print(f"{name}: {len(ts)} workgroups; entries spread {rel[:, 0].max():.2f} us, last epilogue issued at "
          f"{rel[:, 4].max():.2f} us")
    for i, n in enumerate(names):
        print(f"   {n:18s} median {np.median(ph[:, i]):6.2f} us  max {ph[:, i].max():6.2f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--diag", type=int, default=12)
    ap.add_argument("--bdiag", type=int, default=12)
    a = ap.parse_args()
    if a.build:
        from weatherforecast_stgcn_maml_amd import build
        print(build.build(out=LIB, defines=["SMAML_KW_PROBE=1"]))
        return
    os.environ["SMAML_LIB"] = LIB
    import torch

    from weatherforecast_stgcn_maml_amd import _capi, synth
    from weatherforecast_stgcn_maml_amd.adapt import adapt
    from weatherforecast_stgcn_maml_amd.config import CONFIG2
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph

    d = CONFIG2
    P = synth.init_params(22, d, gcn_bias_scale=0.1)
    tr = {k: v for k, v in P.items() if k.startswith(("lstm.", "output_layer."))}
    gcn = {k: v for k, v in P.items() if k not in tr and k.startswith("base_stgcn.conv")}
    lats, lons = synth.region_grid()
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(3200, d.num_nodes, synth.t_total_for(20))
    lib = ctypes.CDLL(LIB)
    lib.smaml_kw_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    buf = np.zeros((1024, 5), np.uint64)
    ctx = _capi.Context(d, 0)
    for name, target in ((f"forward diagonal {a.diag}", a.diag), (f"BPTT diagonal {a.bdiag}", 100 + a.bdiag)):
        assert lib.smaml_kw_probe(target, None, 0) > 0  # arm, zero the records
        adapt(d, feats, ei, gcn, tr, "Moscow", epochs=2, device="cuda:0", ctx=ctx)
        torch.cuda.synchronize()
        khz = lib.smaml_kw_probe(0, buf.ctypes.data, 1024)
        assert khz > 0
        report(name, buf.copy(), 1e6 / khz)
    lib.smaml_kw_probe(-1, None, 0)


if __name__ == "__main__":
    main()
