"""Check of bench.py's cpu_baseline extrapolation: time one full config-2 task on
the CPU port -- (K+1) x B = 6 x 32 = 192 consecutive batch-1 sample-steps of the reference's
per-node nn.LSTM path (oracle.refcpu.ReferencePort) -- and compare the per-step mean with the
short sample bench.py prices a meta-step from. Prints progress every 16 steps, then one JSON line.

Usage: python tools/cpu_extrapolation_check.py [--steps 192] [--sample 6]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=192)
    p.add_argument("--sample", type=int, default=6)
    a = p.parse_args()
    import torch

    from oracle import refcpu
    from weatherforecast_stgcn_maml_amd import synth
    from weatherforecast_stgcn_maml_amd.config import SEED, ModelDims
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph

    d = ModelDims(num_nodes=441, hidden_channels=256)
    lats, lons = synth.region_grid(n_lat=21, n_lon=21)
    ei, _, _ = build_spatial_graph(lats, lons, 4)
    P = synth.init_params(SEED, d)
    feats = synth.make_features(synth.task_seed(0), d.num_nodes, a.steps + d.window_size + d.forecast_horizon + 1)
    port = refcpu.ReferencePort(P, d, ei)

    def xy(i):
        x, y = synth.sample_xy(feats, i)
        return torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(np.ascontiguousarray(y))

    port.step(*xy(0))  # warm
    times = []
    for i in range(a.steps):
        x, y = xy(i)
        t0 = time.perf_counter()
        port.step(x, y)
        times.append(time.perf_counter() - t0)
        if (i + 1) % 16 == 0:
            print(f"{i + 1}/{a.steps} steps, mean {np.mean(times):.3f} s", flush=True)
    t = np.asarray(times)
    out = {"threads": torch.get_num_threads(), "steps": a.steps, "full_task_s": float(t.sum()),
           "mean_s": float(t.mean()), "std_s": float(t.std()), "sample_steps": a.sample,
           "sample_mean_s": float(t[:a.sample].mean()),
           "extrapolation_error": float(t[:a.sample].mean() / t.mean() - 1.0)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
