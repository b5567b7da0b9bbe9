"""Outer meta-training driver mirroring ``train_hybrid_maml_v5.main`` (:187-383) around the
libsmaml meta-step: per epoch, adaptive task sampling (``np.random.choice`` of BATCH_SIZE of
the tasks with probabilities from the per-task loss EMA, :265-280), one meta-step, the EMA
update (:287-292), ``CosineAnnealingWarmRestarts(T_0=10, T_mult=2, eta_min=1e-6)`` per epoch
(:250-252,294), the CSV log ``epoch,meta_loss,learning_rate`` (:256-259,303-304) and the
best / final checkpoints in the reference's dict layout (:306-370).

Task loading from ERA5 (``create_v4_task``, :73-107) is out of scope: callers pass feature
streams (e.g. ``synth.make_features``) resident in HBM.
"""
from __future__ import annotations

import os
import time
from typing import Optional, Sequence

import numpy as np
import torch

from . import checkpoint
from .config import BATCH_SIZE, NUM_EPOCHS, SEED, MamlConfig, ModelDims
from .maml import MetaLearner


class OuterLR:
    """CosineAnnealingWarmRestarts(T_0=10, T_mult=2, eta_min=1e-6) over the outer lr; the
    schedule is held by torch's own scheduler on a one-scalar placeholder optimiser so its
    state_dict is the reference's exactly."""

    def __init__(self, lr: float, T_0=10, T_mult=2, eta_min=1e-6):
        self._p = torch.nn.Parameter(torch.zeros(1))
        self._opt = torch.optim.SGD([self._p], lr=lr)
        self.sched = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(self._opt, T_0=T_0, T_mult=T_mult,
                                                                          eta_min=eta_min)

    @property
    def lr(self) -> float:
        return self._opt.param_groups[0]["lr"]

    def step(self):
        self.sched.step()
        return self.sched.get_last_lr()[0]

    def state_dict(self):
        return self.sched.state_dict()


def meta_train(dims: ModelDims, features: Sequence, edge_index, gcn_full: dict, theta: dict, cfg: MamlConfig,
               epochs: int = NUM_EPOCHS, batch_tasks: int = BATCH_SIZE, koppen_state: Optional[dict] = None,
               log_csv: Optional[str] = None, ckpt_dir: Optional[str] = None, seed: int = SEED,
               device: str = "cuda", verbose: bool = True, dropout=(0.0, 0.0)):
    """Returns (learner, history). ``gcn_full`` holds every non-trainable hybrid tensor
    (conv params + the unused ``base_stgcn.output_layer``) for the checkpoint. ``dropout`` =
    (STGCN dropout_rate, lstm_dropout): the reference trains with (0.2, 0.2); the default (0, 0)
    is the parity setting."""
    rng = np.random.RandomState(seed)
    gcn = {k: v for k, v in gcn_full.items() if k.startswith("base_stgcn.conv")}
    ml = MetaLearner(dims, cfg, gcn, theta, edge_index, device=device, dropout=dropout, dropout_seed=seed)
    feats = [f if torch.is_tensor(f) else torch.from_numpy(np.ascontiguousarray(f)) for f in features]
    feats = [f.to(ml.device, torch.float32).contiguous() for f in feats]
    sched = OuterLR(cfg.outer_lr)
    koppen_state = koppen_state or {"embedding.weight": torch.zeros(31, 8)}
    task_losses: list = []
    best = float("inf")
    hist = []
    if log_csv:
        with open(log_csv, "w") as f:
            f.write("epoch,meta_loss,learning_rate\n")
    n = len(feats)
    loss = float("nan")
    for epoch in range(epochs):
        t0 = time.time()
        if n > batch_tasks and task_losses:
            tot = sum(task_losses)
            probs = np.array(task_losses) / tot if tot > 0 else None
            idx = rng.choice(n, batch_tasks, replace=False, p=probs)
        elif n > batch_tasks:
            idx = rng.choice(n, batch_tasks, replace=False)
        else:
            idx = np.arange(n)
        ml.set_tasks([feats[i] for i in idx], task_ids=idx)
        res = ml.meta_step(lr=sched.lr)
        loss = res.meta_loss
        if len(task_losses) < n:
            task_losses.extend([loss] * (n - len(task_losses)))
        else:
            task_losses = [0.9 * t + 0.1 * loss for t in task_losses]
        lr = sched.step()
        hist.append({"epoch": epoch + 1, "meta_loss": loss, "lr": lr, "tasks": idx.tolist(),
                     "time_s": time.time() - t0})
        if verbose:
            print(f"Epoch {epoch + 1}/{epochs} - Loss: {loss:.4f} - LR: {lr:.6f} - Time: {time.time() - t0:.1f}s")
        if log_csv:
            with open(log_csv, "a") as f:
                f.write(f"{epoch + 1},{loss},{lr}\n")
        if loss < best:
            best = loss
            if ckpt_dir:
                os.makedirs(ckpt_dir, exist_ok=True)
                checkpoint.save(checkpoint.meta_checkpoint(
                    dims, gcn_full, ml.theta, koppen_state, ml.m, ml.v, ml.step, sched.state_dict(), epoch, best,
                    lr=sched.lr, initial_lr=cfg.outer_lr), os.path.join(ckpt_dir, "hybrid_maml_model_v5_best.pt"))
    if ckpt_dir:
        checkpoint.save(checkpoint.meta_checkpoint(
            dims, gcn_full, ml.theta, koppen_state, ml.m, ml.v, ml.step, sched.state_dict(), epochs, best,
            final_loss=loss, lr=sched.lr, initial_lr=cfg.outer_lr),
            os.path.join(ckpt_dir, "hybrid_maml_model_v5_final.pt"))
    return ml, hist
