"""BASELINE config 4 (regional adaptation, adapt_hybrid_v5.py:65-257): one fine-tuning epoch of the
pretrained init on one region -- 960 shuffled batch-1 train steps (fwd + bwd + clip + Adam(L2)),
then the no-grad validation pass over the 240 held-out windows -- timed on one MI355X.

Prints ONE JSON line: sample-steps/s of the train epoch (inputs resident in HBM, the whole epoch
is one smaml_adapt_steps call), the epoch and validation times, and the reference's CPU path
(oracle.refcpu.ReferencePort, batch-1 per-node nn.LSTM loop) timed on a bounded sample of the same
sample-steps on this host. Synthetic ERA5-shaped stream (seed 1000), random-init weights.

Usage: python tools/bench_adapt.py [--epochs 2] [--warmup 1] [--cpu-sample-steps 4]
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
    p.add_argument("--epochs", type=int, default=2, help="timed epochs")
    p.add_argument("--warmup", type=int, default=1, help="untimed epochs")
    p.add_argument("--max-samples", type=int, default=1200)
    p.add_argument("--cpu-sample-steps", type=int, default=4)
    p.add_argument("--region", default="Amazon")
    a = p.parse_args()
    import torch

    from weatherforecast_stgcn_maml_amd import _capi, adapt, params, synth
    from weatherforecast_stgcn_maml_amd.config import SEED, ModelDims
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph

    d = ModelDims(num_nodes=441, hidden_channels=256)
    lats, lons = synth.region_grid(n_lat=21, n_lon=21)
    ei, _, _ = build_spatial_graph(lats, lons, 4)
    P = synth.init_params(SEED, d)
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    gcn = {k: v for k, v in P.items() if k not in names}
    theta = {k: P[k] for k in names}
    T_total = a.max_samples + d.window_size + d.forecast_horizon
    feats = synth.make_features(synth.task_seed(0), d.num_nodes, T_total)
    dev = torch.device("cuda:0")
    ctx = _capi.Context(d, 0)
    ctx.set_graph(ei)
    ctx.set_gcn_params(params.pack(gcn, d, which=1, device=dev))
    th = params.pack(theta, d, which=0, device=dev)
    stream_t = torch.from_numpy(np.ascontiguousarray(feats)).to(dev)
    ctx.set_tasks([stream_t])
    ctx.set_task_ids([0])
    n_all = synth.num_samples(T_total, d.window_size, d.forecast_horizon)
    n_max = min(a.max_samples, n_all)
    n_train = int(0.8 * n_max)
    lr, wd = adapt.climate_optimizer_config(a.region, 0.0006)
    m = torch.zeros_like(th)
    v = torch.zeros_like(th)
    losses = torch.empty(n_train, device=dev)
    stream = _capi.stream_ptr(torch)
    step = 0

    def epoch():
        nonlocal step
        order = adapt.random_sampler_order(n_train).numpy().astype(np.int32)
        lr_dev = torch.full((n_train,), lr, device=dev, dtype=torch.float32)
        ctx.adapt_steps(stream, th, m, v, step, order.reshape(n_train, 1), lr_dev, (0.9, 0.999), 1e-8, wd,
                        adapt.MAX_GRAD_NORM, losses)
        step += n_train

    for _ in range(a.warmup):
        epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.epochs):
        epoch()
    torch.cuda.synchronize()
    t_epoch = (time.perf_counter() - t0) / a.epochs
    loss = float(losses.double().mean().item())
    t0 = time.perf_counter()
    val = adapt.evaluate(ctx, th, list(range(n_train, n_max)), 32)
    torch.cuda.synchronize()
    t_val = time.perf_counter() - t0
    assert np.isfinite(loss) and np.isfinite(val), (loss, val)

    out = {
        "metric": "regional adaptation sample-steps/sec (batch-1 fwd+bwd+clip+Adam, N=441, T=24)",
        "value": n_train / t_epoch,
        "unit": "sample-steps/s",
        "n_gpus": 1,
        "epochs": a.epochs,
        "warmup": a.warmup,
        "ms_per_epoch": t_epoch * 1e3,
        "ms_per_sample_step": t_epoch / n_train * 1e3,
        "val_ms": t_val * 1e3,
        "higher_is_better": True,
        "dtype": "f32",
        "data": "synthetic ERA5-shaped feature stream (numpy PCG64 seed 1000), random-init weights",
        "config": {"workload": f"BASELINE config 4: adaptation epoch of {n_train} shuffled batch-1 train steps "
                               f"+ {n_max - n_train}-window validation, N=441, Hc=256, LSTM 4x128, Adam(L2) "
                               f"lr {lr:g} wd {wd:g} ({a.region})",
                   "train_samples": n_train, "val_samples": n_max - n_train},
        "train_loss": loss,
        "val_loss": val,
    }
    if a.cpu_sample_steps > 0:
        from bench import cpu_baseline
        t_cpu, cores = cpu_baseline(d, a.cpu_sample_steps, P, ei, feats)
        out["cpu_baseline"] = {"value": 1.0 / t_cpu, "unit": "sample-steps/s", "cores": cores, "kind": "port",
                               "sample": f"{a.cpu_sample_steps} batch-1 sample-steps of the reference's per-node "
                                         f"nn.LSTM CPU path at N=441, {t_cpu:.3f} s each"}
        out["vs_cpu_baseline"] = out["value"] * t_cpu
    print(json.dumps(out))


if __name__ == "__main__":
    main()
