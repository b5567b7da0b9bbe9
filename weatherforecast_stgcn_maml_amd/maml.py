"""MAML driver over libsmaml.so (replaces train_hybrid_maml_v5.py:110-184's hot loop).

One ``MetaLearner.meta_step()`` = for every task: K inner SGD steps of B samples
(``inner_loop_v4``, train_hybrid_maml_v5.py:110-141: MSE, backward, clip_grad_norm_(1.0),
SGD lr 0.01), then one B-sample query batch; the meta-gradient (order 1 = first-order,
order 0 = reference semantics where the outer update is a no-op) is summed
over tasks, all-reduced across ranks (RCCL via torch.distributed, one flat buffer),
clipped and applied with AdamW (train_hybrid_maml_v5.py:174-179,245-249) identically
on every rank. The inner loop never returns to Python.

Semantic note (F10): the reference steps its (no-op) outer optimiser every
GRAD_ACCUMULATION_STEPS=2 tasks; here there is one outer step per meta-batch.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _capi, params, synth
from .config import MamlConfig, ModelDims
from .distributed import active, reduce_meta, shard_tasks  # noqa: F401  (shard_tasks re-exported)


def reference_query_start(n_samples: int) -> int:
    """First query sample of a task with ``n_samples`` windows: the reference splits
    ``min(600, len(dataset))`` samples 75/25 into support / query and queries ``query_ds[0]``
    (train_hybrid_maml_v5.py:97-104,162-164)."""
    return int(0.75 * min(600, n_samples))


def query_starts(cfg: MamlConfig, n_samples: Sequence[int], support: Optional[int] = None) -> List[int]:
    """First query sample of each task for ``MetaLearner.default_windows``: the reference split
    (``reference_query_start``) when it lies past the S support samples the inner loop reads
    ((k*B + b) mod S), else S itself, so the query batch never re-uses a support sample (the
    reference, with 15 support samples, never meets this case; a stream shorter than about S/0.75
    samples or S > 450 does). Raises ValueError when the B query samples do not fit the stream."""
    S = support or cfg.support_samples or cfg.inner_steps * cfg.batch
    out = []
    for n in n_samples:
        q0 = max(S, reference_query_start(n))
        if q0 + cfg.batch > n:
            raise ValueError(f"a task stream of {n} samples cannot hold {S} support samples followed by a "
                             f"{cfg.batch}-sample query batch (need >= {S + cfg.batch}; see stream_len_for)")
        out.append(q0)
    return out


def window_table(cfg: MamlConfig, n_tasks: int, support: Optional[int] = None,
                 query_start=None) -> np.ndarray:
    """int32 [(K+1)][tasks][B]: support step k uses samples (k*B + b) mod S (with B=1,
    S=15 this is the reference's 6 epochs x first 15 support samples, :124-127); the
    query batch uses samples q0 .. q0+B-1 (``query_ds[0]`` when B=1, :162-164). ``query_start``:
    one int or one per task (default S; MetaLearner passes ``query_starts`` of its tasks'
    streams)."""
    K, B = cfg.inner_steps, cfg.batch
    S = support or cfg.support_samples or K * B
    q0 = np.broadcast_to(np.asarray(S if query_start is None else query_start, np.int64), (n_tasks,))
    w = np.empty((K + 1, n_tasks, B), np.int32)
    for k in range(K):
        w[k] = ((k * B + np.arange(B)) % S)[None, :]
    w[K] = q0[:, None] + np.arange(B)[None, :]
    return w


def stream_len_for(cfg: MamlConfig, dims: ModelDims, support: Optional[int] = None) -> int:
    """Shortest feature stream whose reference split (``reference_query_start``) puts the query
    batch after the S support samples, with B query samples available. For S > 450 the reference
    split (75 % of at most 600 samples) cannot lie past S; the stream then holds S + B samples and
    ``query_starts`` places the query batch at S."""
    S = support or cfg.support_samples or cfg.inner_steps * cfg.batch
    n = S + cfg.batch
    while reference_query_start(n) < min(S, 450) or n < max(S, reference_query_start(n)) + cfg.batch:
        n += 1
    return synth.t_total_for(n, dims.window_size, dims.forecast_horizon)


KEEP_MARGIN = 8 << 30   # matches api.cpp ensure_keep's free-HBM margin


def task_bytes(dims: ModelDims, cfg: MamlConfig, kept: int) -> int:
    """Device bytes one task holds in a second-order meta-step (api.cpp reserve /
    ensure_so_store / ensure_keep): workspace [F, gcn ping-pong: 3 Hc; Hs, Cs, Gs and their
    tangents: 12 L H per row], the per-step GCN feature cache, and ``kept`` inner steps'
    primal (the last one 5 L H per row: dG + dh; the others 11 L H: Hs, Cs, Gs, dG, dh)."""
    rows = cfg.batch * dims.window_size * dims.num_nodes
    Hc, H, L, K = dims.hidden_channels, dims.lstm_hidden_size, dims.lstm_num_layers, cfg.inner_steps
    f = rows * (3 * Hc + 12 * L * H) + K * rows * Hc
    if kept > 0:
        f += rows * L * H * (5 + 11 * (kept - 1))
    return 4 * f


def plan_task_group(dims: ModelDims, cfg: MamlConfig, n_tasks: int, free_bytes: int) -> int:
    """Tasks per pass of the C driver for a second-order meta-step: the largest group whose
    workspace fits with EVERY inner step's primal kept (tangent-only sweep), balanced over the
    groups it implies; all tasks at once when that already fits (or when nothing would)."""
    if cfg.order != 2 or n_tasks <= 1:
        return n_tasks
    per = task_bytes(dims, cfg, cfg.inner_steps)
    g = max(1, int((free_bytes - KEEP_MARGIN) // per))
    if g >= n_tasks:
        return n_tasks
    ngroups = -(-n_tasks // g)
    return -(-n_tasks // ngroups)


@dataclass
class StepResult:
    losses: torch.Tensor        # [(K+1), tasks] (device); last row = query MSE
    norms: torch.Tensor         # [K, tasks] pre-clip inner grad norms
    meta_loss: float            # sum_tasks query_mse * query_loss_scale (all ranks)
    meta_grad_norm: Optional[float]


class MetaLearner:
    """Holds theta (flat trainable vector), AdamW state and the tasks of this rank."""

    def __init__(self, dims: ModelDims, cfg: MamlConfig, gcn_params: dict, theta: dict,
                 edge_index: np.ndarray, device=None, process_group=None, task_group="auto",
                 dropout=(0.0, 0.0), dropout_seed: int = 0, mem_share: float = 1.0):
        """``task_group``: tasks batched into one pass of the C driver. ``None`` = all of this
        rank's tasks at once; ``"auto"`` (default) = plan_task_group: second-order meta-steps run
        in groups small enough that every inner step's primal stays resident for the sweep.
        The meta-gradient is summed over groups before the all-reduce and outer step.

        ``dropout = (p_gcn, p_lstm)``: train-mode dropout as the reference applies it in its
        inner loop (STGCN ``dropout_rate`` after conv1-3, ``lstm_dropout`` between LSTM layers
        and on the head input), with counter-based masks keyed by
        (``dropout_seed``, meta-step, global task id, inner step, element). (0, 0) = off: the
        reference parity setting.

        ``mem_share``: the fraction of the device's free HBM the "auto" task-group plan may use (several
        processes sharing one GPU, e.g. a multi-rank rehearsal on one device, each plan for their share)."""
        self.mem_share = float(mem_share)
        self.dims = dims
        self.cfg = cfg
        self.task_group = task_group
        self.dropout = (float(dropout[0]), float(dropout[1]))
        self.dropout_seed = int(dropout_seed)
        self.device = torch.device(device or "cuda")
        self.ctx = _capi.Context(dims, self.device.index or 0)
        self.ctx.set_graph(edge_index)
        self.gcn = params.pack(gcn_params, dims, which=1, device=self.device)
        self.ctx.set_gcn_params(self.gcn)
        self.theta = params.pack(theta, dims, which=0, device=self.device)
        P = self.theta.numel()
        # ONE collective per meta-step: the meta-gradient and the query-loss sum share a buffer
        self._reduce = torch.zeros(P + 64, device=self.device)
        self.meta_grad = self._reduce[:P]
        self._qsum = self._reduce[P:P + 1]
        self.m = torch.zeros(P, device=self.device)
        self.v = torch.zeros(P, device=self.device)
        self.step = 0          # outer (AdamW) steps taken
        self.meta_steps = 0    # meta-steps run (any order): keys each meta-step's dropout masks
        self.pg = process_group
        self.tasks: List[torch.Tensor] = []
        self._groups = []
        # HIP events around the per-meta-step all-reduce (bench: the collective's exposed time)
        self.comm_timing = False
        self._comm_ev = []

    # tasks are [t_total, N, 24] float32 feature streams resident in HBM
    def set_tasks(self, features: Sequence, task_ids: Optional[Sequence[int]] = None):
        """``task_ids``: global ids of these tasks (dropout mask keys; default 0..n-1). An empty
        list is allowed (a rank with no task still joins the all-reduce with zeros)."""
        feats = []
        for f in features:
            t = f if torch.is_tensor(f) else torch.from_numpy(np.ascontiguousarray(f))
            feats.append(t.to(self.device, torch.float32).contiguous())
        self.tasks = feats
        self.task_ids = np.asarray(task_ids if task_ids is not None else np.arange(len(feats)), np.int32)
        if not feats:
            self._groups = []
            return
        tg = self.task_group
        if tg == "auto":
            free, _ = torch.cuda.mem_get_info(self.device)
            tg = plan_task_group(self.dims, self.cfg, len(feats), int(free * self.mem_share))
        G = min(tg or len(feats), len(feats))
        self._groups = [(z0, feats[z0:z0 + G]) for z0 in range(0, len(feats), G)]
        self.ctx.set_tasks(self._groups[0][1])
        self.ctx.reserve(G, self.cfg.batch)
        self._mg_part = torch.zeros_like(self.meta_grad) if len(self._groups) > 1 else None

    def default_windows(self) -> np.ndarray:
        """The window table meta_step uses without an explicit one: support samples
        (k*B + b) mod S, query batch from ``query_starts`` (the reference split of each task's
        stream, never inside the support samples)."""
        n = [synth.num_samples(f.shape[0], self.dims.window_size, self.dims.forecast_horizon) for f in self.tasks]
        return window_table(self.cfg, len(self.tasks), query_start=query_starts(self.cfg, n))

    def meta_step(self, windows: Optional[np.ndarray] = None, fast_out=None, sync=True,
                  lr: Optional[float] = None) -> StepResult:
        cfg = self.cfg
        Z = len(self.tasks)
        if windows is None and Z:
            windows = self.default_windows()
        K = cfg.inner_steps
        stream = _capi.stream_ptr(torch)
        if self.dropout != (0.0, 0.0):  # fresh masks every meta-step
            self.ctx.set_dropout(self.dropout[0], self.dropout[1],
                                 (self.dropout_seed * 1000003 + self.meta_steps * 7919 + 1) & 0xFFFFFFFF)
        else:
            self.ctx.set_dropout(0.0, 0.0, 0)
        self.meta_steps += 1
        if Z == 0:  # nothing sharded here: contribute zeros to the reduction
            losses = torch.empty(K + 1, 0, device=self.device)
            norms = torch.empty(max(K, 1), 0, device=self.device)
            self._reduce.zero_()
        elif len(self._groups) == 1:
            self.ctx.set_task_ids(self.task_ids)
            losses = torch.empty(K + 1, Z, device=self.device)
            norms = torch.empty(max(K, 1), Z, device=self.device)
            self.ctx.meta_step(stream, self.theta, cfg.order, K, cfg.batch, windows, cfg.inner_lr,
                               cfg.max_norm, cfg.query_loss_scale,
                               meta_grad=self.meta_grad if cfg.order >= 1 else None,
                               losses=losses, norms=norms, fast_out=fast_out)
        else:
            lparts, nparts = [], []
            for gi, (z0, grp) in enumerate(self._groups):
                n = len(grp)
                lg = torch.empty(K + 1, n, device=self.device)
                ng = torch.empty(max(K, 1), n, device=self.device)
                self.ctx.set_tasks(grp)
                self.ctx.set_task_ids(self.task_ids[z0:z0 + n])
                mg = (self.meta_grad if gi == 0 else self._mg_part) if cfg.order >= 1 else None
                self.ctx.meta_step(stream, self.theta, cfg.order, K, cfg.batch, windows[:, z0:z0 + n],
                                   cfg.inner_lr, cfg.max_norm, cfg.query_loss_scale, meta_grad=mg,
                                   losses=lg, norms=ng, fast_out=fast_out[z0:z0 + n] if fast_out is not None else None)
                if gi > 0 and mg is not None:
                    self.meta_grad.add_(mg)
                lparts.append(lg)
                nparts.append(ng)
            losses = torch.cat(lparts, 1)
            norms = torch.cat(nparts, 1)
        if Z:
            self._qsum.copy_((losses[K].sum() * cfg.query_loss_scale).reshape(1))
        # one all_reduce of [meta_grad | query-loss sum] (just the scalar in reference mode)
        if self.comm_timing and active():
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            reduce_meta(self._reduce if cfg.order >= 1 else self._qsum, self.pg)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._comm_ev.append((e0, e1))
        else:
            reduce_meta(self._reduce if cfg.order >= 1 else self._qsum, self.pg)
        if cfg.order >= 1:
            self.step += 1
            norm_out = torch.empty(1, device=self.device)
            self.ctx.adamw_step(stream, self.theta, self.meta_grad, self.m, self.v, self.step,
                                cfg.outer_lr if lr is None else lr, cfg.outer_betas, cfg.outer_eps, cfg.outer_weight_decay,
                                cfg.outer_max_norm, norm_out)
        else:
            norm_out = None
        if not sync:
            return StepResult(losses, norms, float("nan"), None)
        self.ctx.sync(stream)  # surfaces a timed-out grid-barrier kernel as SmamlError
        return StepResult(losses, norms, float(self._qsum.item()),
                          float(norm_out.item()) if norm_out is not None else None)

    def comm_time_collect(self):
        """(summed ms, count) of the timed all-reduces since the last call: from the end of this rank's
        meta-step work on the stream to the reduced buffer being ready, i.e. the collective plus the
        wait for the slowest rank (synchronises)."""
        torch.cuda.synchronize(self.device)
        ms = sum(e0.elapsed_time(e1) for e0, e1 in self._comm_ev)
        n = len(self._comm_ev)
        self._comm_ev = []
        return ms, n

    def theta_named(self):
        return {k: v.detach().clone() for k, v in params.unpack(self.theta, self.dims, 0).items()}
