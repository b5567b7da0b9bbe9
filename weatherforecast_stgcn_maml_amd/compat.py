"""Reference-signature entry points over libsmaml.so (SURVEY §8b "compat wrapper").

``inner_loop_v4(hybrid_model, koppen_embed, support_ds, device)`` and
``meta_update_v4(hybrid_model, koppen_embed, tasks, device, meta_optimizer)`` keep the
signatures and semantics of train_hybrid_maml_v5.py:110-141 and :144-184: 6 inner epochs
over the first 15 support samples at batch 1 (90 sequential SGD steps, lr 0.01,
clip_grad_norm_(1.0)), query on ``query_ds[0]``, ``meta_loss = sum_tasks MSE_q / 2``, and the
outer update left a no-op exactly as the reference's deep-copy leaves it. All
tasks of a call are batched into the same launches.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from . import params
from .config import (GRAD_ACCUMULATION_STEPS, INNER_BATCH_CAP, INNER_EPOCHS_PER_TASK, INNER_LR,
                     MAX_GRAD_NORM, MamlConfig)
from .dataset import resolve_windows
from .hybrid_model import draw_dropout_seed
from .maml import MetaLearner


def _learner(hybrid_model, edge_index, device, steps, num_nodes):
    dims = hybrid_model.dims(num_nodes)
    cfg = MamlConfig(inner_steps=steps, batch=1, order=0, inner_lr=INNER_LR, max_norm=MAX_GRAD_NORM,
                     query_loss_scale=1.0 / GRAD_ACCUMULATION_STEPS)
    ei = edge_index.detach().cpu().numpy() if torch.is_tensor(edge_index) else np.asarray(edge_index)
    # the reference adapts a train()-mode copy (train_hybrid_maml_v5.py:113,159): its dropout
    # rates apply; every call draws a fresh mask seed from the global torch RNG, as
    # the reference's nn.Dropout calls draw fresh masks
    drop = (float(hybrid_model.base_stgcn.dropout.p), float(hybrid_model.dropout.p))
    seed = draw_dropout_seed() if drop != (0.0, 0.0) else 0
    return MetaLearner(dims, cfg, hybrid_model.named_gcn(), hybrid_model.named_trainable(), ei, device=device,
                       dropout=drop, dropout_seed=seed), dims


def _support_len(windows) -> int:
    """Samples inner_loop_v4 trains on: the first min(15, len(support_ds)) (:124-127)."""
    return min(len(windows), INNER_BATCH_CAP)


def _run(hybrid_model, task_specs, device):
    """task_specs: [(features, support_windows, query_window, edge_index)] sharing one graph and
    one support length (so one inner-step count)."""
    S = _support_len(task_specs[0][1])
    if any(_support_len(sw) != S for _, sw, _, _ in task_specs):
        raise ValueError("tasks batched into one pass must have the same support length")
    K = INNER_EPOCHS_PER_TASK * S
    N = task_specs[0][0].shape[1]
    ml, dims = _learner(hybrid_model, task_specs[0][3], device, K, N)
    ml.set_tasks([f for f, _, _, _ in task_specs])
    w = np.empty((K + 1, len(task_specs), 1), np.int32)
    for z, (_, sw, qw, _) in enumerate(task_specs):
        sw = sw[:S]
        w[:K, z, 0] = [sw[k % S] for k in range(K)]
        w[K, z, 0] = qw
    fast = torch.zeros(len(task_specs), ml.theta.numel(), device=ml.device)
    res = ml.meta_step(windows=w, fast_out=fast)
    return res, fast, dims


def _adapted_copy(hybrid_model, fast_row, dims):
    m = copy.deepcopy(hybrid_model)
    named = params.unpack(fast_row, dims, 0)
    with torch.no_grad():
        for n, p in m.lstm.named_parameters():
            p.copy_(named["lstm." + n])
        m.output_layer.weight.copy_(named["output_layer.weight"])
        m.output_layer.bias.copy_(named["output_layer.bias"])
    return m.train()


def inner_loop_v4(hybrid_model, koppen_embed, support_ds, device):
    feats, windows, ds = resolve_windows(support_ds)
    f = feats.to(device, torch.float32).contiguous()
    res, fast, dims = _run(hybrid_model, [(f, windows, windows[0], ds.edge_index)], device)
    temp_koppen = copy.deepcopy(koppen_embed).train()
    return _adapted_copy(hybrid_model, fast[0], dims), temp_koppen


def meta_update_v4(hybrid_model, koppen_embed, tasks, device, meta_optimizer):
    if meta_optimizer is not None:
        meta_optimizer.zero_grad()
    groups = {}
    for support_ds, query_ds, _stats in tasks:
        if support_ds is None:
            continue
        feats, sw, ds = resolve_windows(support_ds)
        qf, qw, _ = resolve_windows(query_ds)
        if qf is not feats:
            raise ValueError("support and query of a task must share one feature stream")
        ei = ds.edge_index.detach().cpu().numpy() if torch.is_tensor(ds.edge_index) else np.asarray(ds.edge_index)
        # one pass per (graph, support length): tasks in a pass share edge_index and step count
        key = (ei.tobytes(), _support_len(sw))
        groups.setdefault(key, []).append((feats.to(device, torch.float32).contiguous(), sw, qw[0], ei))
    meta_loss = 0.0
    for specs in groups.values():
        res, _, _ = _run(hybrid_model, specs, device)
        meta_loss += float(res.losses[-1].sum().item()) / GRAD_ACCUMULATION_STEPS
    return meta_loss
