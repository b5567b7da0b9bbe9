"""Drop-in for the reference ``model.py`` (``STGCN`` + the PyG ``GCNConv`` it uses).

Same constructor signatures, attribute names and state_dict keys
(``conv{k}.bias``, ``conv{k}.lin.weight``, ``output_layer.{weight,bias}``) as
``model.py:7-52`` with PyG 2.x ``GCNConv``. Compute runs in libsmaml.so (HIP, gfx950);
there is no CPU path.
"""
from __future__ import annotations

import math
import weakref

import numpy as np
import torch
import torch.nn as nn

from . import _capi
from .config import ModelDims

_CTX_CACHE = {}


def _context(dims: ModelDims, device: torch.device):
    if device.type != "cuda":
        raise _capi.SmamlError(-1, "the STGCN-LSTM HIP path needs tensors on a HIP device (cuda)")
    key = (dims, device.index or 0)
    ctx = _CTX_CACHE.get(key)
    if ctx is None:
        ctx = _capi.Context(dims, device.index or 0)
        _CTX_CACHE[key] = ctx
    return ctx


class _GraphMemo:
    """Remembers one edge_index tensor (by identity and autograd version counter, which every in-place
    write to it or to a view of it bumps) together with what was derived from it on the host, so a
    caller that passes the same unchanged tensor every step (train_hybrid_maml_v5.py:129-139) pays
    no device-to-host copy or sync after the first call. Storage swaps (``t.data = other``) are noticed
    through the data pointer; an in-place write through ``t.data`` is invisible to both checks -- pass a
    new tensor (or write without ``.data``) when the graph changes."""

    __slots__ = ("ref", "version", "ptr", "value")

    def __init__(self):
        self.ref = None
        self.version = -1
        self.ptr = 0
        self.value = None

    def get(self, t: torch.Tensor):
        if self.ref is not None and self.ref() is t and t._version == self.version and t.data_ptr() == self.ptr:
            return self.value
        return None

    def put(self, t: torch.Tensor, value):
        self.ref = weakref.ref(t)
        self.version = t._version
        self.ptr = t.data_ptr()  # (`t.data = other` swaps the storage without a version bump)
        self.value = value
        return value


def _set_graph(ctx, edge_index: torch.Tensor):
    memo = ctx.__dict__.setdefault("_ei_memo", _GraphMemo())
    if memo.get(edge_index) is not None and ctx.graph_key is memo.value:
        return
    ei = edge_index.detach().to("cpu", torch.int64).contiguous().numpy()
    key = ei.tobytes()
    if ctx.graph_key != key:
        ctx.set_graph(ei)
    memo.put(edge_index, ctx.graph_key)


class _Linear(nn.Module):
    """PyG ``Linear(in, out, bias=False, weight_initializer='glorot')``."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        a = math.sqrt(6.0 / (in_channels + out_channels))
        nn.init.uniform_(self.weight, -a, a)

    def forward(self, x):  # pragma: no cover - GCNConv drives the fused kernel
        raise NotImplementedError("GCNConv.lin is applied inside the HIP GCN kernel")


class GCNConv(nn.Module):
    """PyG 2.x ``GCNConv(in, out)`` (normalize=True, add self loops, bias). forward
    runs ``smaml_gcn_conv``: rows < num_nodes of the graph aggregate over in-edges
    (symmetric normalisation), all other rows see only their self loop (F3)."""

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin = _Linear(in_channels, out_channels)
        self.bias = nn.Parameter(torch.zeros(out_channels))

    def graph_context(self, x, edge_index):
        """The library context this conv runs in for ``edge_index`` (graph uploaded once per tensor)."""
        memo = self.__dict__.setdefault("_ei_memo", _GraphMemo())
        n_graph = memo.get(edge_index)
        if n_graph is None:  # first call with this edge_index (or it changed): one host sync
            ei = edge_index.detach().to("cpu", torch.int64)
            n_graph = memo.put(edge_index, int(ei.max().item()) + 1 if ei.numel() else 1)
        dims = ModelDims(num_nodes=n_graph, window_size=1, input_channels=max(4, self.in_channels),
                         hidden_channels=max(4, self.out_channels), lstm_hidden_size=32,
                         lstm_num_layers=1, forecast_horizon=1, output_channels=1)
        ctx = _context(dims, x.device)
        _set_graph(ctx, edge_index)
        return ctx

    def forward(self, x, edge_index):
        ctx = self.graph_context(x, edge_index)
        x = x.contiguous().float()
        if torch.is_grad_enabled() and (x.requires_grad or self.lin.weight.requires_grad or self.bias.requires_grad):
            return _GCNConvFn.apply(x, ctx, self.lin.weight, self.bias)
        out = torch.empty(x.shape[0], self.out_channels, device=x.device, dtype=torch.float32)
        ctx.gcn_conv(_capi.stream_ptr(torch), x, self.lin.weight.detach().contiguous(),
                     self.bias.detach().contiguous(), out)
        return out

    def __repr__(self):
        return f"GCNConv({self.in_channels}, {self.out_channels})"


def _conv_backward(lib_ctx, st, x, w, dz, dx, flags=0):
    """smaml_gcn_conv_backward for any out-channel count: its GEMMs take cout in multiples of 4, so a
    ragged cout (e.g. out_channels * forecast_horizon = 3) runs with zero-padded dz columns / W rows,
    whose products are exact zeros (dx unchanged; the padded dW rows and db entries are dropped).
    Returns (dW, db)."""
    cout = w.shape[0]
    c4 = -(-cout // 4) * 4
    if c4 != cout:
        dz = torch.nn.functional.pad(dz, (0, c4 - cout))
        w = torch.nn.functional.pad(w, (0, 0, 0, c4 - cout))
    dwb = torch.empty(w.numel() + c4, device=x.device, dtype=torch.float32)
    lib_ctx.gcn_conv_backward(st, x, w, dz, dx=dx, dwb=dwb, flags=flags)
    return dwb[:w.numel()].view(c4, -1)[:cout], dwb[w.numel():w.numel() + cout]


class _GCNConvFn(torch.autograd.Function):
    """out = A_hat x W^T + b with its backward on the HIP path (smaml_gcn_conv_backward): dx = A_hat^T dz W,
    dW = dz^T (A_hat x), db = sum dz (PyG GCNConv's autograd, model.py:23-26)."""

    @staticmethod
    def forward(fctx, x, lib_ctx, weight, bias):
        w = weight.detach().contiguous()
        out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
        lib_ctx.gcn_conv(_capi.stream_ptr(torch), x, w, bias.detach().contiguous(), out)
        fctx.save_for_backward(x, w)
        fctx.lib_ctx = lib_ctx
        return out

    @staticmethod
    def backward(fctx, gout):
        x, w = fctx.saved_tensors
        dz = gout.contiguous().float()
        need_x = fctx.needs_input_grad[0]
        dx = torch.empty_like(x) if need_x else None
        dw, db = _conv_backward(fctx.lib_ctx, _capi.stream_ptr(torch), x, w, dz, dx)
        return dx, None, dw, db


def _stgcn_run(x, ctxs, dctx, p, seed, num_nodes, params):
    """STGCN.forward (model.py:30-52) in libsmaml: conv1..conv4 each with its ReLU fused into the GCN
    kernel's epilogue (smaml_gcn_conv_ex GCN_RELU), train-mode dropout after each (smaml_dropout,
    counter-based masks; p = 0: none), the last time block through output_layer (smaml_gcn_conv_ex
    GCN_PLAIN: x W^T + b, no aggregation). Returns (out [num_nodes, out*horizon], [x, h1..h4])."""
    st = _capi.stream_ptr(torch)
    hs = [x]
    h = x
    for k in range(4):
        w, b = params[2 * k].detach().contiguous(), params[2 * k + 1].detach().contiguous()
        out = torch.empty(h.shape[0], w.shape[0], device=x.device, dtype=torch.float32)
        ctxs[k].gcn_conv_ex(st, h, w, b, out, flags=_capi.GCN_RELU)
        if p > 0.0:
            dctx.dropout(st, out, p, seed, k)
        hs.append(out)
        h = out
    wo, bo = params[8].detach().contiguous(), params[9].detach().contiguous()
    last = h[-num_nodes:]
    out = torch.empty(num_nodes, wo.shape[0], device=x.device, dtype=torch.float32)
    ctxs[3].gcn_conv_ex(st, last, wo, bo, out, flags=_capi.GCN_PLAIN)
    return out, hs


class _STGCNFn(torch.autograd.Function):
    """STGCN.forward (model.py:30-52) on the HIP path with its backward: conv1..conv4 + ReLU
    (smaml_gcn_conv_ex), train-mode dropout after each (smaml_dropout, counter-based masks), the last
    time block through output_layer (smaml_gcn_conv_ex without aggregation). The backward replays the
    masks on the gradient, applies the ReLU derivative from the saved activations (smaml_relu_mask) and
    runs smaml_gcn_conv_backward per layer."""

    @staticmethod
    def forward(fctx, x, convs, ctxs, dctx, p, seed, num_nodes, *params):
        out, hs = _stgcn_run(x, ctxs, dctx, p, seed, num_nodes, params)
        fctx.save_for_backward(*hs)
        fctx.ctxs, fctx.dctx, fctx.p, fctx.seed, fctx.num_nodes = ctxs, dctx, p, seed, num_nodes
        fctx.ws = [params[2 * k].detach().contiguous() for k in range(4)] + [params[8].detach().contiguous()]
        return out

    @staticmethod
    def backward(fctx, gout):
        st = _capi.stream_ptr(torch)
        hs = fctx.saved_tensors
        N, ctxs, ws = fctx.num_nodes, fctx.ctxs, fctx.ws
        grads = [None] * 10
        h4 = hs[4]
        wo = ws[4]
        dlast = torch.empty(N, h4.shape[1], device=h4.device, dtype=torch.float32)
        grads[8], grads[9] = _conv_backward(ctxs[3], st, h4[-N:], wo, gout.contiguous().float(), dlast,
                                            flags=_capi.GCN_PLAIN)
        g = torch.zeros_like(h4)
        g[-N:] = dlast
        need_x = fctx.needs_input_grad[0]
        for k in range(3, -1, -1):
            if fctx.p > 0.0:
                fctx.dctx.dropout(st, g, fctx.p, fctx.seed, k)  # same masks: d dropout(y) = dropout(d)
            ctxs[k].relu_mask(st, g, hs[k + 1])
            dx = torch.empty_like(hs[k]) if (k > 0 or need_x) else None
            grads[2 * k], grads[2 * k + 1] = _conv_backward(ctxs[k], st, hs[k], ws[k], g, dx)
            g = dx
        return (g if need_x else None, None, None, None, None, None, None, *grads)


def _any_context(device):
    """A context for device-wide helper launches (e.g. smaml_dropout) on ``device``."""
    return _context(ModelDims(num_nodes=1, window_size=1, input_channels=4, hidden_channels=4, lstm_hidden_size=32,
                              lstm_num_layers=1, forecast_horizon=1, output_channels=1), device)


class STGCN(nn.Module):
    """model.py:7-52. ``forward`` (not on the hybrid path) returns the last time block's
    node features through ``output_layer`` as the reference does (model.py:44-52); in
    ``train()`` mode it applies ``self.dropout`` after each of the four conv + ReLU layers
    (model.py:33,36,39,42) with the library's counter-based masks, a fresh seed per call drawn
    from the global torch RNG. With grad enabled it is differentiable (``_STGCNFn``: every conv, the
    ReLUs, the dropout masks and the head run forward and backward in libsmaml), so STGCN trains on
    its own as the reference module does; under no_grad the forward-only path runs."""

    def __init__(self, in_channels, hidden_channels, out_channels=12, window_size=6,
                 forecast_horizon=1, dropout_rate=0.3):
        super().__init__()
        self.window_size = window_size
        self.out_channels = out_channels
        self.forecast_horizon = forecast_horizon
        self.dropout_rate = dropout_rate
        self.conv1 = GCNConv(in_channels, hidden_channels)
        self.conv2 = GCNConv(hidden_channels, hidden_channels)
        self.conv3 = GCNConv(hidden_channels, hidden_channels)
        self.conv4 = GCNConv(hidden_channels, hidden_channels)
        self.dropout = nn.Dropout(p=dropout_rate)
        self.output_layer = nn.Linear(hidden_channels, out_channels * forecast_horizon)

    def _params(self):
        out = []
        for conv in (self.conv1, self.conv2, self.conv3, self.conv4):
            out += [conv.lin.weight, conv.bias]
        return out + [self.output_layer.weight, self.output_layer.bias]

    def forward(self, x, edge_index):
        p = float(self.dropout.p) if self.training else 0.0
        dctx, seed = None, 0
        if p > 0.0:
            from .hybrid_model import draw_dropout_seed
            seed = draw_dropout_seed()
            dctx = _any_context(x.device)
        params = self._params()
        x = x.contiguous().float()
        convs = (self.conv1, self.conv2, self.conv3, self.conv4)
        ctxs = [cv.graph_context(x, edge_index) for cv in convs]
        num_nodes = x.shape[0] // self.window_size
        if torch.is_grad_enabled() and (x.requires_grad or any(q.requires_grad for q in params)):
            out = _STGCNFn.apply(x, convs, ctxs, dctx, p, seed, num_nodes, *params)
        else:  # no_grad: the same launches, nothing saved
            out, _ = _stgcn_run(x, ctxs, dctx, p, seed, num_nodes, params)
        return out.view(num_nodes, self.forecast_horizon, self.out_channels).reshape(-1, self.out_channels)
