"""ctypes binding of ``libsmaml.so`` (C ABI declared in ``include/smaml.h``).

The product path has no CPU fallback: if the library is missing or no HIP device is
present, every compute entry point raises ``SmamlError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SMAML_LIB") or os.path.join(HERE, "libsmaml.so")

# every function include/smaml.h declares (checked by tests/test_capi_cpu.py)
EXPORTS = (
    "smaml_last_error", "smaml_abi_version", "smaml_build_info", "smaml_param_layout", "smaml_graph_ell",
    "smaml_create", "smaml_destroy", "smaml_set_graph", "smaml_set_gcn_params", "smaml_reserve",
    "smaml_workspace_bytes", "smaml_so_kept_steps", "smaml_set_dropout", "smaml_set_task_ids", "smaml_gcn_conv", "smaml_forward", "smaml_set_tasks",
    "smaml_meta_step", "smaml_adamw_step", "smaml_adapt_steps", "smaml_timing", "smaml_timing_collect",
    "smaml_backward", "smaml_gcn_forward", "smaml_lstm_forward", "smaml_lstm_backward", "smaml_head_loss",
    "smaml_clip_sgd", "smaml_inner_loop", "smaml_alloc", "smaml_free", "smaml_comm_unique_id",
    "smaml_comm_init", "smaml_comm_allreduce", "smaml_comm_destroy", "smaml_variant_counts", "smaml_set_option",
    "smaml_dropout", "smaml_sync", "smaml_gcn_conv_ex", "smaml_gcn_conv_backward", "smaml_relu_mask",
    "smaml_adapt_prepare", "smaml_adapt_phases",
)
ABI_VERSION = 7
GCN_RELU, GCN_PLAIN = 1, 2  # smaml_gcn_conv_ex / _backward flags

# kernels.h enum Variant: launch counters per kernel tile configuration (smaml_variant_counts)
VARIANTS = ("fwd", "fwd_drop", "fwd_split", "fwd_img", "fwd_dual", "fwd_dual_kept", "fwd_dual_img", "bwd_big", "bwd_small", "bwd_split",
            "bwd_dual_big", "bwd_dual_big_kept", "bwd_dual_small", "bwd_dual_small_kept", "wgrad", "wgrad_wide", "wgrad_pair",
            "fwd_kw", "bwd_kw", "gcn_dedup", "xg_dedup", "wgrad_dedup", "f_compact")

# api.cpp enum Cat: one kernel per category (the bench's roofline kernel is one symbol)
TIMING_CATEGORIES = ("gcn_layer", "lstm_fwd_step", "lstm_fwd_dual", "head_loss", "head_dh", "lstm_bwd_step",
                     "lstm_bwd_dual", "wgrad", "wgrad_reduce", "misc", "xg_proj", "dg_rowsum",
                     "lstm_fwd_step_wall", "lstm_fwd_dual_wall", "lstm_bwd_step_wall", "lstm_bwd_dual_wall")

ERRORS = {1: "EINVAL", 2: "EHIP", 3: "ENOMEM", 4: "ESTATE", 5: "ENOTIMPL"}


class SmamlError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"smaml error {ERRORS.get(code, code)}: {msg}")
        self.code = code


class Dims(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "num_nodes", "window_size", "input_channels", "hidden_channels", "lstm_hidden_size",
        "lstm_num_layers", "forecast_horizon", "output_channels")]

    @classmethod
    def from_model(cls, d):
        return cls(d.num_nodes, d.window_size, d.input_channels, d.hidden_channels,
                   d.lstm_hidden_size, d.lstm_num_layers, d.forecast_horizon, d.output_channels)


_lock = threading.Lock()
_lib = None

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F32 = ctypes.c_float
PI64 = ctypes.POINTER(ctypes.c_int64)
PI32 = ctypes.POINTER(ctypes.c_int32)
PF32 = ctypes.POINTER(ctypes.c_float)
PDIMS = ctypes.POINTER(Dims)

_SIGS = {
    "smaml_last_error": ([], ctypes.c_char_p),
    "smaml_abi_version": ([], I32),
    "smaml_build_info": ([], ctypes.c_char_p),
    "smaml_param_layout": ([PDIMS, I32, PI64, PI64, I32, PI32, PI64], I32),
    "smaml_graph_ell": ([PI64, I64, I32, PI32, PF32], I32),
    "smaml_create": ([PDIMS, I32, ctypes.POINTER(P)], I32),
    "smaml_destroy": ([P], I32),
    "smaml_set_graph": ([P, PI64, I64], I32),
    "smaml_set_gcn_params": ([P, P], I32),
    "smaml_reserve": ([P, I32, I32], I32),
    "smaml_workspace_bytes": ([P], I64),
    "smaml_so_kept_steps": ([P], I32),
    "smaml_set_dropout": ([P, ctypes.c_float, ctypes.c_float, ctypes.c_uint32], I32),
    "smaml_set_task_ids": ([P, PI32, I32], I32),
    "smaml_gcn_conv": ([P, P, P, I32, I32, P, P, I32, P], I32),
    "smaml_forward": ([P, P, P, ctypes.POINTER(P), I32, P, P], I32),
    "smaml_set_tasks": ([P, I32, ctypes.POINTER(P), PI32], I32),
    "smaml_meta_step": ([P, P, P, I32, I32, I32, PI32, F32, F32, F32, P, P, P, P], I32),
    "smaml_adamw_step": ([P, P, P, P, P, P, I64, I32, F32, F32, F32, F32, F32, F32, P], I32),
    "smaml_adapt_steps": ([P, P, P, P, P, I32, I32, I32, PI32, P, F32, F32, F32, F32, F32, P], I32),
    "smaml_timing": ([P, I32], I32),
    "smaml_backward": ([P, P, P, P, P], I32),
    "smaml_gcn_forward": ([P, P, ctypes.POINTER(P), I32, P], I32),
    "smaml_lstm_forward": ([P, P, P, P, I32, P], I32),
    "smaml_lstm_backward": ([P, P, P, P, P], I32),
    "smaml_head_loss": ([P, P, P, P, ctypes.POINTER(P), I32, P, P, P], I32),
    "smaml_clip_sgd": ([P, P, P, P, I32, F32, F32, P], I32),
    "smaml_inner_loop": ([P, P, P, I32, I32, PI32, F32, F32, P, P, P], I32),
    "smaml_alloc": ([P, I64, ctypes.POINTER(P)], I32),
    "smaml_free": ([P, P], I32),
    "smaml_comm_unique_id": ([ctypes.POINTER(ctypes.c_uint8)], I32),
    "smaml_comm_init": ([P, I32, I32, ctypes.POINTER(ctypes.c_uint8)], I32),
    "smaml_comm_allreduce": ([P, P, P, I64], I32),
    "smaml_comm_destroy": ([P], I32),
    "smaml_timing_collect": ([P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                              PI64, I32], I32),
    "smaml_variant_counts": ([P, PI64, I32, PI32, I32], I32),
    "smaml_set_option": ([P, ctypes.c_char_p, I64], I32),
    "smaml_dropout": ([P, P, P, I64, F32, ctypes.c_uint32, I32], I32),
    "smaml_sync": ([P, P], I32),
    "smaml_gcn_conv_ex": ([P, P, P, I32, I32, P, P, I32, I32, P], I32),
    "smaml_gcn_conv_backward": ([P, P, P, I32, I32, P, I32, P, I32, P, P], I32),
    "smaml_relu_mask": ([P, P, P, P, I64], I32),
    "smaml_adapt_prepare": ([P, P, I32], I32),
    "smaml_adapt_phases": ([P, ctypes.POINTER(ctypes.c_double), I32, PI32, PI64], I32),
}
# smaml_adapt_phases order (api.cpp AdPhases)
ADAPT_PHASES = ("reserve_ms", "cache_alloc_ms", "cache_fill_ms", "steps_ms")


def lib():
    """Load libsmaml.so (raises SmamlError if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise SmamlError(-1, f"{LIB_PATH} not built; run __graft_entry__.build()")
            L = ctypes.CDLL(LIB_PATH)
            L.smaml_abi_version.restype = I32
            if L.smaml_abi_version() != ABI_VERSION:
                raise SmamlError(-1, f"{LIB_PATH} has ABI {L.smaml_abi_version()}, expected {ABI_VERSION}; rebuild")
            for name, (args, res) in _SIGS.items():
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            _lib = L
    return _lib


def build_info() -> str:
    """The library's product form per GEMM family (smaml_build_info)."""
    return lib().smaml_build_info().decode()


def product_forms() -> dict:
    """{GEMM family: 0 = f32 MFMA, 1 = bf16x6 fragment split, 2 = bf16x6 staged split} (build_info())."""
    tail = build_info().split(":", 1)[1]
    return {k: int(v) for k, v in (kv.split("=") for kv in tail.split())}


def check(rc):
    if rc != 0:
        raise SmamlError(rc, lib().smaml_last_error().decode(errors="replace"))


def param_layout(dims, which: int):
    """[(offset, size)] of the flat trainable (which=0) or GCN (which=1) vector + total."""
    L = lib()
    d = Dims.from_model(dims)
    cap = 64
    offs = (ctypes.c_int64 * cap)()
    sizes = (ctypes.c_int64 * cap)()
    cnt = ctypes.c_int32()
    tot = ctypes.c_int64()
    check(L.smaml_param_layout(ctypes.byref(d), which, offs, sizes, cap, ctypes.byref(cnt),
                               ctypes.byref(tot)))
    return [(offs[i], sizes[i]) for i in range(cnt.value)], tot.value


def graph_ell(edge_index: np.ndarray, num_nodes: int):
    L = lib()
    ei = np.ascontiguousarray(edge_index, dtype=np.int64)
    E = ei.shape[1]
    cols = np.zeros((num_nodes, 8), np.int32)
    vals = np.zeros((num_nodes, 8), np.float32)
    check(L.smaml_graph_ell(ei.ctypes.data_as(PI64), E, num_nodes, cols.ctypes.data_as(PI32),
                            vals.ctypes.data_as(PF32)))
    return cols, vals


def ptr(t) -> int:
    return t.data_ptr()


def _ptrs(ts):
    return (P * len(ts))(*[ptr(t) for t in ts])


def comm_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0), to ship to the other ranks."""
    buf = (ctypes.c_uint8 * 128)()
    check(lib().smaml_comm_unique_id(buf))
    return bytes(buf)


def stream_ptr(torch_mod):
    return torch_mod.cuda.current_stream().cuda_stream


class Context:
    """Owns one ``smaml_ctx`` (one GPU, one host thread)."""

    def __init__(self, dims, device: int = 0):
        self.dims = dims
        self._L = lib()
        self._h = P()
        self._d = Dims.from_model(dims)
        check(self._L.smaml_create(ctypes.byref(self._d), int(device), ctypes.byref(self._h)))
        self.device = device
        # A/B runs: SMAML_OPTIONS="key=value,key=value" applies smaml_set_option knobs to every context
        for kv in filter(None, os.environ.get("SMAML_OPTIONS", "").split(",")):
            k, _, v = kv.partition("=")
            self.set_option(k.strip(), int(v))
        self._keep = []
        self.graph_key = None

    def close(self):
        if self._h:
            self._L.smaml_destroy(self._h)
            self._h = P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- setup
    def set_graph(self, edge_index: np.ndarray):
        ei = np.ascontiguousarray(edge_index, dtype=np.int64)
        check(self._L.smaml_set_graph(self._h, ei.ctypes.data_as(PI64), ei.shape[1]))
        self.graph_key = ei.tobytes()

    def set_gcn_params(self, flat):
        self._gcn = flat
        check(self._L.smaml_set_gcn_params(self._h, ptr(flat)))

    def reserve(self, tasks, batch):
        check(self._L.smaml_reserve(self._h, int(tasks), int(batch)))

    def workspace_bytes(self):
        return int(self._L.smaml_workspace_bytes(self._h))

    def so_kept_steps(self):
        return int(self._L.smaml_so_kept_steps(self._h))

    def set_dropout(self, p_gcn, p_lstm, seed):
        check(self._L.smaml_set_dropout(self._h, float(p_gcn), float(p_lstm), int(seed) & 0xFFFFFFFF))

    def set_task_ids(self, ids):
        a = np.ascontiguousarray(ids, dtype=np.int32)
        check(self._L.smaml_set_task_ids(self._h, a.ctypes.data_as(PI32), a.size))

    # --- compute
    def gcn_conv(self, stream, x, weight, bias, out):
        check(self._L.smaml_gcn_conv(self._h, stream, ptr(x), x.shape[0], x.shape[1], ptr(weight),
                                     ptr(bias), weight.shape[0], ptr(out)))

    def gcn_conv_ex(self, stream, x, weight, bias, out, flags=0):
        check(self._L.smaml_gcn_conv_ex(self._h, stream, ptr(x), x.shape[0], x.shape[1], ptr(weight), ptr(bias),
                                        weight.shape[0], int(flags), ptr(out)))

    def gcn_conv_backward(self, stream, x, weight, dz, dx=None, dwb=None, flags=0):
        check(self._L.smaml_gcn_conv_backward(self._h, stream, ptr(x), x.shape[0], x.shape[1], ptr(weight),
                                              weight.shape[0], ptr(dz), int(flags),
                                              ptr(dx) if dx is not None else None,
                                              ptr(dwb) if dwb is not None else None))

    def relu_mask(self, stream, g, h):
        check(self._L.smaml_relu_mask(self._h, stream, ptr(g), ptr(h), g.numel()))

    def forward(self, stream, theta, xs, pred, feats=None):
        arr = (P * len(xs))(*[ptr(x) for x in xs])
        check(self._L.smaml_forward(self._h, stream, ptr(theta), arr, len(xs), ptr(pred),
                                    ptr(feats) if feats is not None else None))

    def set_tasks(self, feats):
        arr = (P * len(feats))(*[ptr(f) for f in feats])
        tt = (ctypes.c_int32 * len(feats))(*[int(f.shape[0]) for f in feats])
        self._tasks = list(feats)
        check(self._L.smaml_set_tasks(self._h, len(feats), arr, tt))

    def meta_step(self, stream, theta, order, steps, batch, windows: np.ndarray, inner_lr, max_norm,
                  query_scale, meta_grad=None, losses=None, norms=None, fast_out=None):
        w = np.ascontiguousarray(windows, dtype=np.int32)
        check(self._L.smaml_meta_step(
            self._h, stream, ptr(theta), int(order), int(steps), int(batch), w.ctypes.data_as(PI32),
            float(inner_lr), float(max_norm), float(query_scale),
            ptr(meta_grad) if meta_grad is not None else None,
            ptr(losses) if losses is not None else None,
            ptr(norms) if norms is not None else None,
            ptr(fast_out) if fast_out is not None else None))

    def adapt_steps(self, stream, theta, m, v, step0, windows: np.ndarray, lr_dev, betas, eps, wd, max_norm,
                    losses):
        w = np.ascontiguousarray(windows, dtype=np.int32)
        check(self._L.smaml_adapt_steps(self._h, stream, ptr(theta), ptr(m), ptr(v), int(step0), w.shape[0],
                                        w.shape[1], w.ctypes.data_as(PI32), ptr(lr_dev), float(betas[0]),
                                        float(betas[1]), float(eps), float(wd), float(max_norm), ptr(losses)))

    def adapt_prepare(self, stream, batch=1):
        """Workspace + per-window feature cache for adapt_steps, allocated and touched now (no compute)."""
        check(self._L.smaml_adapt_prepare(self._h, stream, int(batch)))

    def adapt_phases(self):
        """{phase: ms} of the last adapt_steps call (+ 'windows_filled_per_step')."""
        ms = (ctypes.c_double * len(ADAPT_PHASES))()
        n, filled = ctypes.c_int32(), ctypes.c_int64()
        check(self._L.smaml_adapt_phases(self._h, ms, len(ADAPT_PHASES), ctypes.byref(n), ctypes.byref(filled)))
        out = {k: ms[i] for i, k in enumerate(ADAPT_PHASES[:n.value])}
        out["windows_filled_per_step"] = filled.value
        return out

    def backward(self, stream, theta, dpred, grad):
        check(self._L.smaml_backward(self._h, stream, ptr(theta), ptr(dpred), ptr(grad)))

    def gcn_forward(self, stream, xs, feats):
        check(self._L.smaml_gcn_forward(self._h, stream, _ptrs(xs), len(xs), ptr(feats)))

    def lstm_forward(self, stream, theta, feats, hT):
        check(self._L.smaml_lstm_forward(self._h, stream, ptr(theta), ptr(feats), int(feats.shape[0]), ptr(hT)))

    def lstm_backward(self, stream, theta, dhT, grad):
        check(self._L.smaml_lstm_backward(self._h, stream, ptr(theta), ptr(dhT), ptr(grad)))

    def head_loss(self, stream, theta, hT, pred, ys=None, loss=None, dpred=None):
        check(self._L.smaml_head_loss(self._h, stream, ptr(theta), ptr(hT), _ptrs(ys) if ys is not None else None,
                                      int(hT.shape[0]), ptr(pred), ptr(loss) if loss is not None else None,
                                      ptr(dpred) if dpred is not None else None))

    def clip_sgd(self, stream, theta, grad, ntasks, lr, max_norm, norms=None):
        check(self._L.smaml_clip_sgd(self._h, stream, ptr(theta), ptr(grad), int(ntasks), float(lr),
                                     float(max_norm), ptr(norms) if norms is not None else None))

    def sync(self, stream):
        """Synchronise the stream; raises SmamlError if a grid-barrier kernel timed out."""
        check(self._L.smaml_sync(self._h, stream))

    def inner_loop(self, stream, theta, steps, batch, windows: np.ndarray, inner_lr, max_norm, fast_out,
                   losses=None, norms=None):
        w = np.ascontiguousarray(windows, dtype=np.int32)
        check(self._L.smaml_inner_loop(self._h, stream, ptr(theta), int(steps), int(batch), w.ctypes.data_as(PI32),
                                       float(inner_lr), float(max_norm), ptr(fast_out),
                                       ptr(losses) if losses is not None else None,
                                       ptr(norms) if norms is not None else None))

    def alloc(self, nbytes: int) -> int:
        out = P()
        check(self._L.smaml_alloc(self._h, int(nbytes), ctypes.byref(out)))
        return out.value

    def free(self, p: int):
        check(self._L.smaml_free(self._h, P(p)))

    def comm_init(self, rank: int, world: int, uid: bytes):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self._L.smaml_comm_init(self._h, int(rank), int(world), buf))

    def comm_allreduce(self, stream, buf):
        check(self._L.smaml_comm_allreduce(self._h, stream, ptr(buf), buf.numel()))

    def comm_destroy(self):
        check(self._L.smaml_comm_destroy(self._h))

    def timing(self, enable: bool):
        check(self._L.smaml_timing(self._h, 1 if enable else 0))

    def timing_collect(self):
        n = len(TIMING_CATEGORIES)
        ms = (ctypes.c_double * n)()
        fl = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        check(self._L.smaml_timing_collect(self._h, ms, fl, cnt, n))
        return {name: {"ms": ms[i], "flops": fl[i], "launches": cnt[i]}
                for i, name in enumerate(TIMING_CATEGORIES)}

    def variant_counts(self, reset: bool = False):
        """{variant: launches} since the last reset (host counters, no sync)."""
        n = len(VARIANTS)
        buf = (ctypes.c_int64 * n)()
        cnt = ctypes.c_int32()
        check(self._L.smaml_variant_counts(self._h, buf, n, ctypes.byref(cnt), 1 if reset else 0))
        assert cnt.value == n, (cnt.value, n)
        return {name: int(buf[i]) for i, name in enumerate(VARIANTS)}

    def dropout(self, stream, x, p, seed, layer):
        check(self._L.smaml_dropout(self._h, stream, ptr(x), x.numel(), float(p), int(seed) & 0xFFFFFFFF, int(layer)))

    def set_option(self, key: str, value: int):
        check(self._L.smaml_set_option(self._h, key.encode(), int(value)))

    def adamw_step(self, stream, theta, grad, m, v, step, lr, betas, eps, wd, max_norm, norm_out=None):
        check(self._L.smaml_adamw_step(self._h, stream, ptr(theta), ptr(grad), ptr(m), ptr(v),
                                       theta.numel(), int(step), float(lr), float(betas[0]),
                                       float(betas[1]), float(eps), float(wd), float(max_norm),
                                       ptr(norm_out) if norm_out is not None else None))
