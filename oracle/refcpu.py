"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU (torch fp32) restatement of the reference hot path. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / CPU baseline. The product path
(``weatherforecast_stgcn_maml_amd``) never imports it.

Pinned against golden vectors produced by running the reference modules themselves
(``tests/golden/make_fixtures.py``; see ``tests/test_oracle_golden.py``). The PyG
``GCNConv`` arithmetic is third-party (torch_geometric, unvendored, version unpinned,
absent from this image): it is restated from PyG 2.x's published ``gcn_norm`` +
``propagate`` and is "parity unpinned" at that boundary.

What each function follows:
  * ``gcn_conv``            PyG 2.x GCNConv (called at model.py:23-26, hybrid_model.py:65-74)
  * ``stgcn_features``      hybrid_model.py:60-78 (no_grad GCN x4 + ReLU, dropout p=0)
  * ``stgcn_forward``       model.py:30-52 (STGCN's own forward: last time block + output_layer)
  * ``lstm_stack``          nn.LSTM(batch_first) semantics, gates [i,f,g,o] (hybrid_model.py:42-49,93-102)
  * ``hybrid_forward``      hybrid_model.py:80-117 (F3, F4 layouts)
  * ``mse``                 nn.MSELoss on the F4-permuted rows (train_hybrid_maml_v5.py:119,133)
  * ``clip_coef``           torch.nn.utils.clip_grad_norm_ (train_hybrid_maml_v5.py:135-138)
  * ``inner_loop``          train_hybrid_maml_v5.py:110-141 (SGD lr 0.01, batch of B samples)
  * ``meta_step``           train_hybrid_maml_v5.py:144-184 (+ FO / second-order meta-grad)
  * ``ReferencePort``       op-for-op mirror (per-node nn.LSTM loop, batch 1) for CPU timing
  * ``regional_eval``       validate_hybrid_v5.py:189-237,337-358 (denormalised per-variable metrics),
                            pinned to validateAdapted itself run on synthetic data (cfg*_validate.npz)
  * ``climate_lr``          adaptive_scheduler.py:29-55 (ClimateAwareLRScheduler.step)
  * ``adapt_reference``     adapt_hybrid_v5.py:152-231 (adaptModel's fine-tune + validation),
                            pinned to adaptModel itself run on synthetic data (cfg4_adapt.npz)
  * ``Dropout``             train-mode dropout (hybrid_model.py:67,70,73,108; nn.LSTM dropout :47)
                            with the HIP path's counter-based masks (kernels.h drop_keep),
                            restated here so masks agree bit for bit; the reference draws its
                            masks from torch's RNG, so only p = 0 is pinned to the reference
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- dropout masks
_M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    """lowbias32 on uint64 arrays holding 32-bit values (kernels.h mix32)."""
    x = x & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


def drop_site(seed: int, kind: int, step: int, layer: int) -> np.uint64:
    k = np.uint64(((kind << 24) ^ (step << 8) ^ layer) & 0xFFFFFFFF)
    return _mix32(np.uint64(seed & 0xFFFFFFFF) ^ _mix32(k))


def drop_keep(site, idx: np.ndarray, p: float) -> np.ndarray:
    """bool mask: element idx (uint64) of a site is kept iff
    (mix32(site ^ lo(idx) ^ hi(idx) * 0x9E3779B9) >> 8) >= round(p * 2^24)."""
    idx = np.asarray(idx, dtype=np.uint64)
    thr = np.uint64(min(int(round(p * 16777216.0)), 16777216))
    hi = ((idx >> np.uint64(32)) * np.uint64(0x9E3779B9)) & _M32
    h = _mix32(np.uint64(site) ^ (idx & _M32) ^ hi)
    return (h >> np.uint64(8)) >= thr


class Dropout:
    """Masks of one forward pass (meta-step seed, inner step) for one task (global id)."""

    def __init__(self, seed: int, p_gcn: float, p_lstm: float, task: int, step: int):
        self.seed, self.p_gcn, self.p_lstm, self.task, self.step = seed, p_gcn, p_lstm, task, step

    def _apply(self, x: torch.Tensor, kind: int, layer: int, base: int, p: float) -> torch.Tensor:
        if p <= 0.0:
            return x
        idx = np.uint64(base) + np.arange(x.numel(), dtype=np.uint64)
        keep = torch.from_numpy(drop_keep(drop_site(self.seed, kind, self.step, layer), idx, p))
        return x * keep.view(x.shape).to(x.dtype) * (1.0 / (1.0 - p))

    def gcn(self, h: torch.Tensor, layer: int, b: int, B: int) -> torch.Tensor:
        """h [T*N, Hc] of sample b of the batch after conv layer+1 (layer 0..2)."""
        return self._apply(h, 1, layer, (self.task * B + b) * h.numel(), self.p_gcn)

    def lstm(self, out: torch.Tensor, layer: int) -> torch.Tensor:
        """out [M, T, H] (sequences m = b*N + n) of LSTM layer `layer` fed to layer+1; the
        element order of the masks is [t][m][unit]."""
        M, T, H = out.shape
        tm = out.permute(1, 0, 2).contiguous()
        return self._apply(tm, 2, layer, self.task * T * M * H, self.p_lstm).permute(1, 0, 2)

    def head(self, hT: torch.Tensor) -> torch.Tensor:
        return self._apply(hT, 3, 0, self.task * hT.numel(), self.p_lstm)


# ----------------------------------------------------------------------------- GCN
def gcn_conv(x: torch.Tensor, edge_index: torch.Tensor, weight: torch.Tensor,
             bias: torch.Tensor) -> torch.Tensor:
    """PyG 2.x GCNConv: add_remaining_self_loops over all x rows, deg at target,
    norm = d_s^-1/2 d_t^-1/2, out = index_add(target, (x W^T)[source] * norm) + bias."""
    n = x.shape[0]
    ei = edge_index.to(torch.long)
    keep = ei[0] != ei[1]
    loop = torch.arange(n, dtype=torch.long)
    row = torch.cat([ei[0][keep], loop])
    col = torch.cat([ei[1][keep], loop])
    w = torch.ones(row.numel(), dtype=x.dtype)
    deg = torch.zeros(n, dtype=x.dtype).scatter_add_(0, col, w)
    dinv = deg.pow(-0.5)
    dinv = dinv.masked_fill(torch.isinf(dinv), 0.0)
    norm = dinv[row] * w * dinv[col]
    xw = x @ weight.t()
    out = torch.zeros(n, weight.shape[0], dtype=x.dtype).index_add_(0, col, xw[row] * norm[:, None])
    return out + bias


def stgcn_features(x: torch.Tensor, edge_index: torch.Tensor, P: Dict[str, torch.Tensor],
                   drop: "Dropout" = None, b: int = 0, B: int = 1):
    h = x
    for k in range(1, 5):
        h = F.relu(gcn_conv(h, edge_index, P[f"base_stgcn.conv{k}.lin.weight"],
                            P[f"base_stgcn.conv{k}.bias"]))
        if drop is not None and k < 4:
            h = drop.gcn(h, k - 1, b, B)
    return h


def stgcn_forward(x: torch.Tensor, edge_index: torch.Tensor, P: Dict[str, torch.Tensor], dims,
                  drop: "Dropout" = None) -> torch.Tensor:
    """model.STGCN.forward (model.py:30-52): conv1..conv4 + ReLU, dropout after EACH of the four
    (train mode; drop = masks of kind 1, layers 0..3), last time block (x[-N:]), output_layer,
    view(N, Hf, C).reshape(-1, C)."""
    h = x
    for k in range(1, 5):
        h = F.relu(gcn_conv(h, edge_index, P[f"base_stgcn.conv{k}.lin.weight"], P[f"base_stgcn.conv{k}.bias"]))
        if drop is not None:
            h = drop.gcn(h, k - 1, 0, 1)
    N = h.shape[0] // dims.window_size
    out = h[-N:] @ P["base_stgcn.output_layer.weight"].t() + P["base_stgcn.output_layer.bias"]
    return out.view(N, dims.forecast_horizon, dims.output_channels).reshape(-1, dims.output_channels)


# ----------------------------------------------------------------------------- LSTM
def lstm_stack(seq: torch.Tensor, P: Dict[str, torch.Tensor], layers: int, drop: "Dropout" = None):
    """seq [B, T, C] -> top-layer h_T [B, H]; h0 = c0 = 0 (drop: masks between layers)."""
    Bn, T, _ = seq.shape
    inp = seq
    for l in range(layers):
        Wih, Whh = P[f"lstm.weight_ih_l{l}"], P[f"lstm.weight_hh_l{l}"]
        b = P[f"lstm.bias_ih_l{l}"] + P[f"lstm.bias_hh_l{l}"]
        H = Whh.shape[1]
        xp = inp @ Wih.t()
        h = torch.zeros(Bn, H, dtype=seq.dtype)
        c = torch.zeros(Bn, H, dtype=seq.dtype)
        outs = []
        for t in range(T):
            g = xp[:, t] + h @ Whh.t() + b
            i, f, gg, o = g.chunk(4, dim=1)
            i, f, gg, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(gg), torch.sigmoid(o)
            c = f * c + i * gg
            h = o * torch.tanh(c)
            outs.append(h)
        inp = torch.stack(outs, dim=1)
        if drop is not None and l < layers - 1:
            inp = drop.lstm(inp, l)
    return inp[:, -1]


def hybrid_forward(P: Dict[str, torch.Tensor], x: torch.Tensor, edge_index: torch.Tensor,
                   dims, feats: torch.Tensor = None) -> torch.Tensor:
    """x [T*N, 24] (time-major rows) -> pred [N*Hf, C] (rows n*Hf + h)."""
    T, N = dims.window_size, dims.num_nodes
    if feats is None:
        with torch.no_grad():
            feats = stgcn_features(x, edge_index, P)
    seq = feats.view(T, N, -1).permute(1, 0, 2)
    hT = lstm_stack(seq, P, dims.lstm_num_layers)
    pred = hT @ P["output_layer.weight"].t() + P["output_layer.bias"]
    return pred.view(N, dims.forecast_horizon, dims.output_channels).reshape(-1, dims.output_channels)


def batched_forward(P, feats_list: Sequence[torch.Tensor], dims, drop: "Dropout" = None) -> List[torch.Tensor]:
    """Same as ``hybrid_forward`` for several samples at once (sequences stacked)."""
    T, N = dims.window_size, dims.num_nodes
    seq = torch.cat([f.view(T, N, -1).permute(1, 0, 2) for f in feats_list], dim=0)
    hT = lstm_stack(seq, P, dims.lstm_num_layers, drop)
    if drop is not None:
        hT = drop.head(hT)
    pred = hT @ P["output_layer.weight"].t() + P["output_layer.bias"]
    pred = pred.view(len(feats_list), N * dims.forecast_horizon, dims.output_channels)
    return list(pred)


def mse(pred: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """nn.MSELoss (mean) row by row; pred rows are [node][horizon], y rows
    [horizon][node] (F4) -- compared as they stand, exactly as the reference does."""
    return ((pred - y) ** 2).mean()


def clip_coef(grads: Sequence[torch.Tensor], max_norm: float):
    norms = torch.stack([g.norm(2) for g in grads])
    total = norms.norm(2)
    return torch.clamp(max_norm / (total + 1e-6), max=1.0), total


# ----------------------------------------------------------------------------- MAML
TRAINABLE_PREFIXES = ("lstm.", "output_layer.")


def trainable_names(P) -> List[str]:
    return [k for k in P if k.startswith(TRAINABLE_PREFIXES)]


def to_torch(P: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)).clone() for k, v in P.items()}


class TaskData:
    """A task's feature stream and graph; samples are windows (dataset.py:30-48)."""

    def __init__(self, features: np.ndarray, edge_index: np.ndarray, dims):
        self.features = torch.from_numpy(np.ascontiguousarray(features))
        self.edge_index = torch.from_numpy(np.ascontiguousarray(edge_index)).long()
        self.dims = dims
        self._feat_cache = {}

    def xy(self, i: int):
        W, Hf, N = self.dims.window_size, self.dims.forecast_horizon, self.dims.num_nodes
        x = self.features[i:i + W].reshape(W * N, -1)
        y = self.features[i + W + 1:i + W + 1 + Hf, :, :12].reshape(Hf * N, 12)
        return x, y

    def gcn(self, i: int, P):
        if i not in self._feat_cache:
            x, _ = self.xy(i)
            with torch.no_grad():
                self._feat_cache[i] = stgcn_features(x, self.edge_index, P)
        return self._feat_cache[i]


def batch_loss(Pt: Dict[str, torch.Tensor], Pg: Dict[str, torch.Tensor], task: TaskData,
               idx: Sequence[int], drop: "Dropout" = None):
    """Mean over the B samples of the per-sample MSE (SURVEY F9 definition)."""
    P = dict(Pg)
    P.update(Pt)
    if drop is None:
        feats = [task.gcn(i, Pg) for i in idx]
    else:
        with torch.no_grad():
            feats = [stgcn_features(task.xy(i)[0], task.edge_index, Pg, drop, b, len(idx)) for b, i in enumerate(idx)]
    preds = batched_forward(P, feats, task.dims, drop)
    losses = torch.stack([mse(p, task.xy(i)[1]) for p, i in zip(preds, idx)])
    return losses.mean(), preds


def support_schedule(step: int, batch: int, support: int) -> List[int]:
    """Samples used by inner step ``step``: ``(step*B + b) mod S``. With B=1, S=15 this
    is the reference's 6 epochs x first 15 support samples (train_hybrid_maml_v5.py:124-127)."""
    return [(step * batch + b) % support for b in range(batch)]


def inner_loop(Pt, Pg, task: TaskData, steps: int, batch: int, support: int, lr: float,
               max_norm: float, create_graph: bool = False, record=None, dropout=None):
    """dropout = (seed, p_gcn, p_lstm, global task id) or None."""
    names = list(Pt.keys())
    params = [Pt[k] for k in names]
    for k in range(steps):
        idx = support_schedule(k, batch, support)
        cur = dict(zip(names, params))
        drop = Dropout(dropout[0], dropout[1], dropout[2], dropout[3], k) if dropout else None
        loss, _ = batch_loss(cur, Pg, task, idx, drop)
        grads = torch.autograd.grad(loss, params, create_graph=create_graph)
        coef, total = clip_coef(grads, max_norm)
        if record is not None:
            record.append((float(loss.detach()), float(total.detach()), float(coef.detach())))
        params = [p - lr * coef * g for p, g in zip(params, grads)]
        if not create_graph:
            params = [p.detach().requires_grad_(True) for p in params]
    return dict(zip(names, params))


def meta_step(Pt0: Dict[str, torch.Tensor], Pg, tasks: Sequence[TaskData], query_idx,
              steps: int, batch: int, support: int, lr: float, max_norm: float,
              order: int, query_scale: float = 0.5, dropout=None, task_ids=None):
    """Returns dict(meta_loss, query_losses, meta_grad (per name, summed over tasks),
    step_records, adapted (per task)). dropout = (seed, p_gcn, p_lstm): masks of inner step k
    keyed (seed, task_ids[j], k), the query batch's (seed, task_ids[j], steps)."""
    names = list(Pt0.keys())
    meta_grad = {k: torch.zeros_like(v) for k, v in Pt0.items()}
    qlosses, records, adapted_all = [], [], []
    for j, task in enumerate(tasks):
        theta0 = [Pt0[k].detach().clone().requires_grad_(True) for k in names]
        rec = []
        tid = task_ids[j] if task_ids is not None else j
        dk = (dropout[0], dropout[1], dropout[2], tid) if dropout else None
        adapted = inner_loop(dict(zip(names, theta0)), Pg, task, steps, batch, support, lr,
                             max_norm, create_graph=(order == 2), record=rec, dropout=dk)
        qdrop = Dropout(dropout[0], dropout[1], dropout[2], tid, steps) if dropout else None
        qloss, _ = batch_loss(adapted, Pg, task, query_idx, qdrop)
        scaled = qloss * query_scale
        if order == 2:
            g = torch.autograd.grad(scaled, theta0)
        elif order == 1:
            g = torch.autograd.grad(scaled, [adapted[k] for k in names])
        else:
            g = [torch.zeros_like(t) for t in theta0]
        for k, gi in zip(names, g):
            meta_grad[k] += gi.detach()
        qlosses.append(float(qloss))
        records.append(rec)
        adapted_all.append({k: v.detach() for k, v in adapted.items()})
    meta_loss = sum(q * query_scale for q in qlosses)
    return dict(meta_loss=meta_loss, query_losses=qlosses, meta_grad=meta_grad,
                step_records=records, adapted=adapted_all)


def adamw_step(params, grads, state, lr, betas=(0.9, 0.999), eps=1e-8, wd=1e-4,
               max_norm=1.0):
    """clip_grad_norm_ then torch.optim.AdamW (decoupled wd), in place; fp32."""
    names = list(grads.keys())
    coef, _ = clip_coef([grads[k] for k in names], max_norm)
    b1, b2 = betas
    state["step"] = state.get("step", 0) + 1
    t = state["step"]
    for k in names:
        g = grads[k] * coef
        m = state.setdefault("m_" + k, torch.zeros_like(g))
        v = state.setdefault("v_" + k, torch.zeros_like(g))
        params[k].mul_(1 - lr * wd)
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        params[k].addcdiv_(m, denom, value=-lr / bc1)
    return params


# ----------------------------------------------------------------------------- CPU port
class ReferencePort:
    """Op-for-op mirror of the reference's inner step for CPU timing: PyG-semantics GCN x4
    under no_grad, a per-node ``nn.LSTM`` loop (hybrid_model.py:93-102), Linear head,
    MSELoss, backward, clip_grad_norm_(1.0), SGD(lr=0.01) -- batch 1."""

    def __init__(self, P: Dict[str, np.ndarray], dims, edge_index: np.ndarray):
        self.dims = dims
        H, L = dims.lstm_hidden_size, dims.lstm_num_layers
        self.lstm = torch.nn.LSTM(dims.hidden_channels, H, L, batch_first=True)
        self.head = torch.nn.Linear(H, dims.head_out)
        with torch.no_grad():
            for name, p in self.lstm.named_parameters():
                p.copy_(torch.from_numpy(P["lstm." + name]))
            self.head.weight.copy_(torch.from_numpy(P["output_layer.weight"]))
            self.head.bias.copy_(torch.from_numpy(P["output_layer.bias"]))
        self.Pg = {k: torch.from_numpy(v) for k, v in P.items() if k.startswith("base_stgcn")}
        self.edge_index = torch.from_numpy(np.asarray(edge_index)).long()
        params = list(self.lstm.parameters()) + list(self.head.parameters())
        self.params = params
        self.opt = torch.optim.SGD(params, lr=0.01)
        self.crit = torch.nn.MSELoss()

    def step(self, x: torch.Tensor, y: torch.Tensor) -> float:
        d = self.dims
        self.opt.zero_grad()
        with torch.no_grad():
            feats = stgcn_features(x, self.edge_index, self.Pg)
        N = feats.shape[0] // d.window_size
        seq = feats.view(d.window_size, N, -1).permute(1, 0, 2)
        outs = []
        for n in range(N):
            o, _ = self.lstm(seq[n:n + 1])
            outs.append(o[0, -1, :])
        pred = self.head(torch.stack(outs, 0))
        pred = pred.view(N, d.forecast_horizon, d.output_channels).reshape(-1, d.output_channels)
        loss = self.crit(pred, y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.params, max_norm=1.0)
        self.opt.step()
        return float(loss)


# ----------------------------------------------------------------------------- evaluation
def regional_eval(P: Dict[str, torch.Tensor], features: np.ndarray, edge_index, stats, dims, num_samples: int = 3):
    """validate_hybrid_v5.validateAdapted's metric path (validate_hybrid_v5.py:189-237,337-358):
    no-grad forward of the first min(3, len) windows, sample means (numpy, fp32), reshape both as
    [Hf, N, 12] (the F4 pairing), node means, denormalise variables 0-5 with stats, MSE / MAE per
    variable, average without sp."""
    d = dims
    T, Hf, N = d.window_size, d.forecast_horizon, d.num_nodes
    n = min(num_samples, features.shape[0] - T - Hf)
    ei = torch.as_tensor(np.asarray(edge_index)).long()
    preds, trues = [], []
    for i in range(n):
        x, y = TaskData(features, ei.numpy(), d).xy(i)
        with torch.no_grad():
            preds.append(hybrid_forward(P, x, ei, d).numpy())
        trues.append(y.numpy())
    y_pred = np.mean(preds, axis=0).reshape(Hf, N, 12).mean(axis=1)
    y_true = np.mean(trues, axis=0).reshape(Hf, N, 12).mean(axis=1)
    mean, std = np.array(stats["mean"]), np.array(stats["std"])
    names = ["u10", "v10", "t2m", "d2m", "sp", "tp"]
    res, tot, cnt = {}, 0.0, 0
    for v, name in enumerate(names):
        t = y_true[:, v] * std[v] + mean[v]
        p = y_pred[:, v] * std[v] + mean[v]
        res[name] = {"mse": np.mean((p - t) ** 2), "mae": np.mean(np.abs(p - t))}
        if name != "sp":
            tot += res[name]["mse"]
            cnt += 1
    res["average_mse"] = tot / cnt
    return res


# ----------------------------------------------------------------------------- adaptation
def climate_lr(region_name, epoch_idx, base_lr, epoch_loss):
    """adaptive_scheduler.ClimateAwareLRScheduler.step (adaptive_scheduler.py:29-55) after
    ``epoch_idx`` (1-based) epochs; base_lr already includes the climate factor of
    create_climate_optimizer, the multiplier is applied again as the reference does."""
    mult = 0.9 if region_name in ("Indonesia", "Thailand", "QueensAustralia") else (
        1.1 if region_name in ("Moscow", "NorthSiberia", "Afghanistan") else 1.0)
    prog = (epoch_idx - 1) % 5 / 5
    lr = base_lr * mult * 0.5 * (1 + np.cos(np.pi * prog))
    if epoch_loss is not None and epoch_idx > 3:
        if epoch_loss > 1.0:
            lr *= 1.1
        elif epoch_loss < 0.2:
            lr *= 0.95
    return lr


def adapt_reference(Pt, Pg, task: TaskData, region_name: str, epochs: int, max_samples: int = 1200,
                    base_lr: float = 0.0006, dropout=None, orders=None):
    """adapt_hybrid_v5.adaptModel's fine-tuning loop (adapt_hybrid_v5.py:152-231): batch-1
    samples in DataLoader(shuffle=True) order (a real torch DataLoader draws it, as PyG's
    loader does), MSE, backward, clip_grad_norm_(1.0), torch.optim.Adam(lr, weight_decay) from
    create_climate_optimizer, scheduler per epoch, then the validation MSE. Returns (params,
    epoch_losses, lrs, val_loss, step_losses). dropout = (seed, p_gcn, p_lstm): train-step masks
    keyed by the global step index (task id 0). orders: optional per-epoch permutations."""
    n_all = task.features.shape[0] - task.dims.window_size - task.dims.forecast_horizon
    n_max = min(max_samples, n_all)
    n_train = int(0.8 * n_max)
    zone_mult = 0.9 if region_name in ("Indonesia", "Thailand", "QueensAustralia") else (
        1.1 if region_name in ("Moscow", "NorthSiberia", "Afghanistan") else 1.0)
    wd = 1e-5 if zone_mult == 0.9 else (5e-5 if zone_mult == 1.1 else 1e-4)
    lr0 = base_lr * zone_mult
    names = list(Pt.keys())
    leaves = [Pt[k].detach().clone().requires_grad_(True) for k in names]
    opt = torch.optim.Adam(leaves, lr=lr0, weight_decay=wd)
    epoch_losses, lrs = [], []
    gstep = 0
    loader = torch.utils.data.DataLoader(range(n_train), batch_size=1, shuffle=True)
    step_losses = []
    for ep in range(epochs):
        order = list(orders[ep]) if orders is not None else [int(b) for b in loader]
        ls = []
        lrs.append(opt.param_groups[0]["lr"])
        for i in order:
            opt.zero_grad()
            drop = Dropout(dropout[0], dropout[1], dropout[2], 0, gstep) if dropout else None
            gstep += 1
            loss, _ = batch_loss(dict(zip(names, leaves)), Pg, task, [i], drop)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(leaves, max_norm=1.0)
            opt.step()
            ls.append(float(loss.detach()))
        avg = sum(ls) / len(ls)
        epoch_losses.append(avg)
        step_losses.append(ls)
        new_lr = climate_lr(region_name, ep + 1, lr0, avg)
        for pg in opt.param_groups:
            pg["lr"] = new_lr
    with torch.no_grad():
        vals = [float(batch_loss(dict(zip(names, leaves)), Pg, task, [i])[0]) for i in range(n_train, n_max)]
    return (dict(zip(names, [l.detach() for l in leaves])), epoch_losses, lrs, sum(vals) / max(len(vals), 1),
            step_losses)
