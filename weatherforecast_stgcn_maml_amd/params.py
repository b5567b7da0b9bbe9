"""Flat parameter vectors (layout owned by the C ABI: ``smaml_param_layout``).

theta (which=0): the 18 trainable tensors (lstm.* then output_layer.*) in state_dict
order -- the tensors ``HybridSTGCN_LSTM.get_trainable_parameters`` returns
(hybrid_model.py:119-124) and the only ones that receive gradients.
gcn (which=1): base_stgcn.conv{1..4}.{bias, lin.weight} (frozen on the hot path).
Offsets are padded to 64 floats; pads stay zero.
"""
from __future__ import annotations

from functools import lru_cache

import numpy as np
import torch

from . import _capi, synth


@lru_cache(maxsize=None)
def _layout(dims, which):
    specs = synth.trainable_param_specs(dims) if which == 0 else [
        s for s in synth.gcn_param_specs(dims) if s[0].startswith("base_stgcn.conv")]
    offs, total = _capi.param_layout(dims, which)
    assert len(offs) == len(specs)
    out = []
    for (name, shape), (off, size) in zip(specs, offs):
        assert int(np.prod(shape)) == size, (name, shape, size)
        out.append((name, tuple(shape), int(off)))
    return tuple(out), int(total)


def trainable_layout(dims):
    return _layout(dims, 0)


def gcn_layout(dims):
    return _layout(dims, 1)


def trainable_count(dims) -> int:
    return sum(int(np.prod(s)) for _, s, _ in trainable_layout(dims)[0])


def pack(named, dims, which=0, device=None, out=None):
    """dict name -> tensor/ndarray  ->  flat float32 tensor (padded layout)."""
    lay, total = _layout(dims, which)
    if out is None:
        out = torch.zeros(total, dtype=torch.float32, device=device)
    dst, src = [], []
    for name, shape, off in lay:
        v = named[name]
        if not torch.is_tensor(v):
            v = torch.from_numpy(np.ascontiguousarray(v))
        n = int(np.prod(shape))
        dst.append(out[off:off + n])
        src.append(v.reshape(-1).to(out.device, torch.float32))
    torch._foreach_copy_(dst, src)  # one multi-tensor launch on a device (the module API packs per forward)
    return out


def unpack(flat, dims, which=0):
    """flat tensor -> dict name -> view (same storage)."""
    lay, _ = _layout(dims, which)
    res = {}
    for name, shape, off in lay:
        n = int(np.prod(shape))
        res[name] = flat[off:off + n].view(shape)
    return res
