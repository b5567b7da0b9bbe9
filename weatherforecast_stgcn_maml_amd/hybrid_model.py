"""Drop-in for the reference ``hybrid_model.py`` (``HybridSTGCN_LSTM``).

Constructor signature, attributes (``base_stgcn``, ``lstm``, ``output_layer``,
``dropout``, ``forecast_horizon``, ``out_channels``, ``lstm_hidden_size``), methods
(``extract_base_features``, ``forward``, ``get_trainable_parameters``,
``freeze_base_model``, ``unfreeze_base_model``) and state_dict keys follow
``hybrid_model.py:6-134``. ``forward`` runs the whole STGCN-LSTM forward in libsmaml.so:
GCN x4 (f32 products on the MFMA pipe, F3 semantics), the 4-layer LSTM batched over nodes (the reference's
per-node loop, F6, is one batched recurrence here), head. No CPU fallback.

With grad enabled, ``forward`` is a ``torch.autograd.Function`` (``_HybridFn``): its backward
is ``smaml_backward`` (head, BPTT, weight gradients on the GPU), so unmodified callers --
``loss.backward()``, ``clip_grad_norm_``, ``torch.optim.*`` as in ``inner_loop_v4``
(train_hybrid_maml_v5.py:110-141) or ``adaptModel`` (adapt_hybrid_v5.py:168-203) -- drive
the HIP path. Gradients reach the LSTM and head only (the reference computes the GCN under
``no_grad``, F2). One forward/backward pair may be in flight per model shape: a second forward
before the backward ends the first one's saved activations (the backward then raises).

In ``train()`` mode the forward applies the reference's dropout sites (STGCN ``dropout`` after
conv1-3 inside ``extract_base_features``, hybrid_model.py:67,70,73; ``nn.LSTM``'s inter-layer
dropout, :42-49; the head-input dropout, :108) with the library's counter-based masks; every
call draws a fresh mask seed from the global torch RNG (as ``nn.Dropout`` draws its masks), and
the backward reuses the forward's masks. ``eval()`` (or p = 0) runs without dropout.
For whole meta-steps use ``weatherforecast_stgcn_maml_amd.maml`` (run entirely inside the
library).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _capi, params
from .config import ModelDims
from .model import _context, _set_graph


def draw_dropout_seed() -> int:
    """One 32-bit mask seed from the global torch RNG (a train-mode forward draws one)."""
    return int(torch.empty((), dtype=torch.int64).random_().item()) & 0xFFFFFFFF


def _forward(lib_ctx, theta, xs, pred, drop, feats=None):
    """smaml_forward, with train-mode dropout (p_gcn, p_lstm, seed) set around it (the masks are
    captured by the forward and reused by the following smaml_backward)."""
    if drop is not None:
        lib_ctx.set_task_ids([0])
        lib_ctx.set_dropout(*drop)
    try:
        lib_ctx.forward(_capi.stream_ptr(torch), theta, xs, pred, feats)
    finally:
        if drop is not None:
            lib_ctx.set_dropout(0.0, 0.0, 0)


class _HybridFn(torch.autograd.Function):
    """pred = HybridSTGCN_LSTM(x) with d pred / d (LSTM, head) from ``smaml_backward``."""

    @staticmethod
    def forward(fctx, x, lib_ctx, dims, theta, names, drop, *tparams):
        pred = torch.empty(dims.num_nodes * dims.forecast_horizon, dims.output_channels, device=x.device)
        _forward(lib_ctx, theta, [x], pred, drop)
        fctx.lib_ctx, fctx.dims, fctx.theta, fctx.names = lib_ctx, dims, theta, names
        return pred

    @staticmethod
    def backward(fctx, gpred):
        grad = torch.empty_like(fctx.theta)
        fctx.lib_ctx.backward(_capi.stream_ptr(torch), fctx.theta, gpred.contiguous().float(), grad)
        g = params.unpack(grad, fctx.dims)
        return (None, None, None, None, None, None, *[g[n] for n in fctx.names])


class LSTMParams(nn.Module):
    """Parameter container with ``nn.LSTM``'s names, shapes and init
    (``weight_ih_l{k}`` [4H, in], ``weight_hh_l{k}`` [4H, H], ``bias_ih_l{k}``,
    ``bias_hh_l{k}``; U(+-1/sqrt(H))). The recurrence itself runs in the HIP library."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True, dropout=0.0,
                 bidirectional=False):
        super().__init__()
        if bidirectional:
            raise ValueError("bidirectional LSTM is not part of the reference path")
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.num_layers = num_layers
        self.batch_first = batch_first
        self.dropout = dropout
        self.bidirectional = False
        G = 4 * hidden_size
        for l in range(num_layers):
            cin = input_size if l == 0 else hidden_size
            self.register_parameter(f"weight_ih_l{l}", nn.Parameter(torch.empty(G, cin)))
            self.register_parameter(f"weight_hh_l{l}", nn.Parameter(torch.empty(G, hidden_size)))
            self.register_parameter(f"bias_ih_l{l}", nn.Parameter(torch.empty(G)))
            self.register_parameter(f"bias_hh_l{l}", nn.Parameter(torch.empty(G)))
        a = 1.0 / math.sqrt(hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -a, a)

    def flatten_parameters(self):
        """No-op (called at train_hybrid_maml_v5.py:212, adapt_hybrid_v5.py:125)."""

    def forward(self, *args, **kwargs):
        raise NotImplementedError("LSTMParams holds weights; HybridSTGCN_LSTM.forward runs the recurrence")


class HybridSTGCN_LSTM(nn.Module):
    def __init__(self, base_stgcn, lstm_hidden_size=64, lstm_num_layers=2, lstm_dropout=0.2,
                 out_channels=12, forecast_horizon=8, freeze_base=True):
        super().__init__()
        self.forecast_horizon = forecast_horizon
        self.out_channels = out_channels
        self.lstm_hidden_size = lstm_hidden_size
        self.base_stgcn = base_stgcn
        if freeze_base:
            for p in self.base_stgcn.parameters():
                p.requires_grad = False
        base_hidden_channels = self.base_stgcn.conv1.out_channels
        self.lstm = LSTMParams(input_size=base_hidden_channels, hidden_size=lstm_hidden_size,
                               num_layers=lstm_num_layers, batch_first=True,
                               dropout=lstm_dropout if lstm_num_layers > 1 else 0.0)
        self.output_layer = nn.Linear(lstm_hidden_size, out_channels * forecast_horizon)
        self.dropout = nn.Dropout(lstm_dropout)

    # ------------------------------------------------------------------ helpers
    def dims(self, num_nodes: int) -> ModelDims:
        b = self.base_stgcn
        return ModelDims(num_nodes=num_nodes, window_size=b.window_size,
                         input_channels=b.conv1.in_channels, hidden_channels=b.conv1.out_channels,
                         lstm_hidden_size=self.lstm_hidden_size,
                         lstm_num_layers=self.lstm.num_layers,
                         forecast_horizon=self.forecast_horizon, output_channels=self.out_channels)

    def named_trainable(self):
        sd = {}
        for n, p in self.lstm.named_parameters():
            sd["lstm." + n] = p.detach()
        sd["output_layer.weight"] = self.output_layer.weight.detach()
        sd["output_layer.bias"] = self.output_layer.bias.detach()
        return sd

    def named_gcn(self):
        b = self.base_stgcn
        out = {}
        for k in range(1, 5):
            conv = getattr(b, f"conv{k}")
            out[f"base_stgcn.conv{k}.bias"] = conv.bias.detach()
            out[f"base_stgcn.conv{k}.lin.weight"] = conv.lin.weight.detach()
        return out

    def _drop(self):
        """(p_gcn, p_lstm, seed) of a train-mode forward, None in eval mode or at p = 0."""
        p_gcn = float(self.base_stgcn.dropout.p)
        p_lstm = float(self.dropout.p)
        if not self.training or (p_gcn <= 0.0 and p_lstm <= 0.0):
            return None
        return (p_gcn, p_lstm, draw_dropout_seed())

    def _prepare(self, x, edge_index):
        if x.device.type != "cuda":
            raise _capi.SmamlError(-1, "HybridSTGCN_LSTM.forward runs on a HIP device only")
        T = self.base_stgcn.window_size
        if x.shape[0] % T:
            raise ValueError(f"x has {x.shape[0]} rows, not a multiple of window_size={T}")
        dims = self.dims(x.shape[0] // T)
        ctx = _context(dims, x.device)
        _set_graph(ctx, edge_index)
        gflat, fresh = self._packed(1, self._gcn_params(), dims, x.device)
        if fresh or getattr(ctx, "_gcn", None) is not gflat:  # another model may share the context
            ctx.set_gcn_params(gflat)
        theta, _ = self._packed(0, self._trainable_params(), dims, x.device)
        return ctx, dims, theta

    def _gcn_params(self):
        b = self.base_stgcn
        out = []
        for k in range(1, 5):
            conv = getattr(b, f"conv{k}")
            out += [(f"base_stgcn.conv{k}.bias", conv.bias), (f"base_stgcn.conv{k}.lin.weight", conv.lin.weight)]
        return out

    def _packed(self, which, named, dims, device):
        """The flat (padded) parameter vector of `named` on `device`, packed into one cached buffer. It is
        re-packed on every call (one multi-tensor copy into the same buffer), so writes that autograd does
        not see (``p.data.copy_(...)``, ``p.data -= lr * g``, numpy arrays aliasing a parameter) are always
        picked up, with or without grad. Returns (flat, changed?): changed is True when a parameter object
        was replaced, its storage moved or it was written in place through autograd's version counter
        (optimizer steps, load_state_dict) -- always True with grad enabled (the backward differentiates at
        this vector) -- and tells callers that hand the buffer to the library by pointer to re-register it."""
        cache = self.__dict__.setdefault("_pack_cache", {})
        objs = [p for _, p in named]
        key = [(p._version, p.data_ptr()) for p in objs]
        ent = cache.get(which)
        same = (not torch.is_grad_enabled() and ent is not None and ent["device"] == device
                and len(ent["objs"]) == len(objs) and all(a is b for a, b in zip(ent["objs"], objs))
                and ent["key"] == key)
        total = (params.trainable_layout(dims) if which == 0 else params.gcn_layout(dims))[1]
        reuse = ent["flat"] if ent is not None and ent["device"] == device and ent["flat"].numel() == total else None
        flat = params.pack({n: p.detach() for n, p in named}, dims, which=which, device=device, out=reuse)
        cache[which] = {"device": device, "objs": objs, "key": key, "flat": flat}
        return flat, not same

    def invalidate_packed(self):
        """Drop the packed parameter vectors (the next forward allocates and packs them afresh). Every
        forward re-packs anyway, so this only releases the buffers."""
        self.__dict__.pop("_pack_cache", None)

    # ------------------------------------------------------------------ module API
    def extract_base_features(self, x, edge_index):
        """hybrid_model.py:60-78 -> [T*N, hidden_channels]."""
        ctx, dims, theta = self._prepare(x, edge_index)
        x = x.contiguous().float()
        pred = torch.empty(dims.num_nodes * dims.forecast_horizon, dims.output_channels, device=x.device)
        feats = torch.empty(x.shape[0], dims.hidden_channels, device=x.device)
        _forward(ctx, theta, [x], pred, self._drop(), feats)
        return feats

    def _trainable_params(self):
        named = [("lstm." + n, p) for n, p in self.lstm.named_parameters()]
        named += [("output_layer.weight", self.output_layer.weight), ("output_layer.bias", self.output_layer.bias)]
        return named

    def forward(self, x, edge_index):
        """hybrid_model.py:80-117 -> [N*forecast_horizon, out_channels] (rows n*Hf + h)."""
        ctx, dims, theta = self._prepare(x, edge_index)
        x = x.contiguous().float()
        named = self._trainable_params()
        drop = self._drop()
        if torch.is_grad_enabled() and any(p.requires_grad for _, p in named):
            return _HybridFn.apply(x, ctx, dims, theta, [n for n, _ in named], drop, *[p for _, p in named])
        pred = torch.empty(dims.num_nodes * dims.forecast_horizon, dims.output_channels, device=x.device)
        _forward(ctx, theta, [x], pred, drop)
        return pred

    def get_trainable_parameters(self):
        trainable = []
        trainable.extend(self.lstm.parameters())
        trainable.extend(self.output_layer.parameters())
        return trainable

    def freeze_base_model(self):
        for p in self.base_stgcn.parameters():
            p.requires_grad = False

    def unfreeze_base_model(self):
        for p in self.base_stgcn.parameters():
            p.requires_grad = True
