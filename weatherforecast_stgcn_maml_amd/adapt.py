"""Regional adaptation (BASELINE config 4) over libsmaml.so.

Mirrors ``adapt_hybrid_v5.adaptModel`` (adapt_hybrid_v5.py:65-271): a 1,200-sample cap split
80/20 into train/validation (:152-159), 15 epochs of shuffled batch-1 fine-tuning — forward,
MSE, backward, ``clip_grad_norm_(1.0)``, ``torch.optim.Adam`` with the climate learning rate
and L2 weight decay (:168-203) — the ``ClimateAwareLRScheduler`` stepped once per epoch on
the epoch's mean loss (:208), a no-grad validation MSE (:216-231) and the adapted checkpoint
(:240-257). Each epoch's steps run inside the library (``smaml_adapt_steps``); Python only
draws the shuffle order and steps the scheduler. Data loading from ERA5 (:30-62) is out of
scope: callers pass a feature stream.

``ClimateAwareLRScheduler`` / ``create_climate_optimizer`` are restated from
adaptive_scheduler.py:7-94 (host-side scalars).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import _capi, params, synth
from .config import MAX_GRAD_NORM, ModelDims

TROPICAL = ("Indonesia", "Thailand", "QueensAustralia")
COLD = ("Moscow", "NorthSiberia", "Afghanistan")
CLIMATE_MULT = {"tropical": 0.9, "temperate": 1.0, "cold": 1.1}
CLIMATE_WD = {"tropical": 1e-5, "temperate": 1e-4, "cold": 5e-5}


def climate_zone(region_name: str) -> str:
    if region_name in TROPICAL:
        return "tropical"
    if region_name in COLD:
        return "cold"
    return "temperate"


def climate_optimizer_config(region_name: str, base_lr: float = 0.0006):
    """(lr, weight_decay) of create_climate_optimizer (adaptive_scheduler.py:68-94)."""
    z = climate_zone(region_name)
    return base_lr * CLIMATE_MULT[z], CLIMATE_WD[z]


class ClimateAwareLRScheduler:
    """adaptive_scheduler.py:7-66: cosine with 5-epoch cycles times the climate multiplier,
    nudged by the epoch loss after epoch 3."""

    def __init__(self, region_name: str, base_lr: float = 0.0006):
        self.region_name = region_name
        self.base_lr = base_lr
        self.current_epoch = 0
        self.lr_multiplier = CLIMATE_MULT[climate_zone(region_name)]

    def step(self, epoch_loss: Optional[float] = None) -> float:
        self.current_epoch += 1
        cycle_length = 5
        cycle_progress = (self.current_epoch - 1) % cycle_length / cycle_length
        cosine_factor = 0.5 * (1 + np.cos(np.pi * cycle_progress))
        lr = self.base_lr * self.lr_multiplier * cosine_factor
        if epoch_loss is not None and self.current_epoch > 3:
            if epoch_loss > 1.0:
                lr *= 1.1
            elif epoch_loss < 0.2:
                lr *= 0.95
        return lr


def random_sampler_order(n: int) -> torch.Tensor:
    """The order a ``DataLoader(ds, batch_size=1, shuffle=True)`` (adapt_hybrid_v5.py:179; PyG's
    loader is torch's) yields in one epoch, drawing from the global torch RNG as it does: the
    iterator first draws its ``_base_seed`` (one int64), then ``RandomSampler`` draws its own seed
    (one int64) and runs ``randperm`` on a generator seeded with it. This reproduces the
    reference's order for its first epoch, and for every epoch only when the adaptation is
    dropout-free: ``adaptModel`` trains in train mode, where each step's ``nn.Dropout`` also draws
    from the global RNG, so from epoch 2 its shuffle depends on draws this path does not make.
    Parity with train-mode adaptation therefore replays recorded orders (``adapt(orders=...)``)."""
    torch.empty((), dtype=torch.int64).random_()  # _BaseDataLoaderIter._base_seed
    seed = int(torch.empty((), dtype=torch.int64).random_().item())
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randperm(n, generator=g)


@dataclass
class AdaptResult:
    theta: torch.Tensor
    epoch_losses: List[float] = field(default_factory=list)
    lrs: List[float] = field(default_factory=list)
    val_loss: float = float("nan")
    n_train: int = 0
    n_val: int = 0


def adapt(dims: ModelDims, features, edge_index, gcn: dict, theta: dict, region_name: str, epochs: int = 15,
          max_samples: int = 1200, train_frac: float = 0.8, base_lr: float = 0.0006, device="cuda",
          val_batch: int = 32, ctx: Optional[_capi.Context] = None, dropout=(0.0, 0.0),
          dropout_seed: int = 0, orders=None) -> AdaptResult:
    """``dropout`` = (STGCN dropout_rate, lstm_dropout) of the train-mode steps (the reference
    adapts in train mode: (0.2, 0.2)); validation runs without dropout (eval mode).
    ``orders``: optional per-epoch sample permutations of the training windows (default: drawn
    from the global torch RNG as the reference's shuffling DataLoader draws them)."""
    dev = torch.device(device)
    ctx = ctx or _capi.Context(dims, dev.index or 0)
    ei = edge_index.detach().cpu().numpy() if torch.is_tensor(edge_index) else np.asarray(edge_index)
    ctx.set_graph(ei)
    gflat = params.pack(gcn, dims, which=1, device=dev)
    ctx.set_gcn_params(gflat)
    th = params.pack(theta, dims, which=0, device=dev)
    stream_t = features if torch.is_tensor(features) else torch.from_numpy(np.ascontiguousarray(features))
    stream_t = stream_t.to(dev, torch.float32).contiguous()
    ctx.set_tasks([stream_t])
    n_all = synth.num_samples(stream_t.shape[0], dims.window_size, dims.forecast_horizon)
    n_max = min(max_samples, n_all)
    n_train = int(train_frac * n_max)
    lr0, wd = climate_optimizer_config(region_name, base_lr)
    sched = ClimateAwareLRScheduler(region_name, lr0)
    m = torch.zeros_like(th)
    v = torch.zeros_like(th)
    res = AdaptResult(theta=th, n_train=n_train, n_val=n_max - n_train)
    stream = _capi.stream_ptr(torch)
    lr = lr0
    step = 0
    losses = torch.empty(max(n_train, 1), device=dev)
    ctx.set_task_ids([0])
    ctx.set_dropout(dropout[0], dropout[1], dropout_seed)
    ctx.adapt_prepare(stream, 1)  # workspace + feature cache before the first epoch (setup, no compute)
    for _ in range(epochs):
        ctx.set_dropout(dropout[0], dropout[1], dropout_seed)  # masks keyed by the global step index
        ep = len(res.epoch_losses)
        order = np.asarray(orders[ep] if orders is not None else random_sampler_order(n_train).numpy(), np.int32)
        assert order.shape == (n_train,), order.shape
        lr_dev = torch.full((n_train,), lr, device=dev, dtype=torch.float32)
        ctx.adapt_steps(stream, th, m, v, step, order.reshape(n_train, 1), lr_dev, (0.9, 0.999), 1e-8, wd,
                        MAX_GRAD_NORM, losses)
        step += n_train
        avg = float(losses[:n_train].double().mean().item())
        res.epoch_losses.append(avg)
        res.lrs.append(lr)
        lr = sched.step(avg)
    ctx.set_dropout(0.0, 0.0, 0)
    res.val_loss = evaluate(ctx, th, list(range(n_train, n_max)), val_batch)
    return res


def evaluate(ctx: _capi.Context, theta: torch.Tensor, sample_ids, batch: int = 32) -> float:
    """Mean per-sample MSE over the given windows of task 0 (no gradients, no dropout)."""
    ctx.set_dropout(0.0, 0.0, 0)
    total, n = 0.0, 0
    stream = _capi.stream_ptr(torch)
    for i in range(0, len(sample_ids), batch):
        chunk = sample_ids[i:i + batch]
        w = np.asarray(chunk, np.int32).reshape(1, 1, len(chunk))
        loss = torch.empty(1, 1, device=theta.device)
        ctx.meta_step(stream, theta, 0, 0, len(chunk), w, 0.0, 1.0, 1.0, losses=loss)
        total += float(loss.item()) * len(chunk)
        n += len(chunk)
    return total / max(n, 1)
