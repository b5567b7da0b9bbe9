"""Robustness of the hot path's bookkeeping kernels and of the fused GCN's shape guard (round 4).

* The grid-barrier kernels (k_inner_sgd: clip_grad_norm_ + SGD, train_hybrid_maml_v5.py:135-139;
  k_sweep_update: the second-order sweep's per-parameter update) bound every wait: a grid that can
  never be co-resident (the ``barrier_oversize`` debug knob) ends in bounded time with SMAML_EHIP
  instead of a hang, the barrier state is reset, and the next launch is correct again.
* The two-launch form of both kernels (``grid_barrier`` 0) is bitwise equal to the fused one.
* The fused GCN stack (k_gcn_mlp) with fewer than 17 input channels (layer 1 still walks two
  zero-padded 16-k image steps) matches the per-layer path and the oracle (hybrid_model.py:60-78).
"""
import time

import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import _capi, params, synth
from weatherforecast_stgcn_maml_amd.config import CONFIG2, MamlConfig, ModelDims
from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

from test_gpu_parity import DEV, grid_edges, rel, split

pytestmark = pytest.mark.gpu


def _clip_sgd_ref(theta, grad, lr, max_norm):
    """torch.nn.utils.clip_grad_norm_ + SGD on each task row (fp64 norm, as the kernel)."""
    out = theta.clone()
    norms = []
    for z in range(theta.shape[0]):
        n = float(torch.linalg.vector_norm(grad[z].double()))
        c = min(1.0, max_norm / (n + 1e-6))
        out[z] = theta[z] - lr * (grad[z] * c)
        norms.append(n)
    return out, norms


def test_grid_barrier_timeout_reports_error_and_recovers():
    d = CONFIG2
    ctx = _capi.Context(d, 0)
    P = _capi.param_layout(d, 0)[1]
    Z = 3
    g = torch.Generator().manual_seed(5)
    theta0 = torch.randn(Z, P, generator=g).to(DEV)
    grad = (torch.randn(Z, P, generator=g) * 0.01).to(DEV)
    grad[1] *= 1000.0  # task 1 clipped, the others not
    st = _capi.stream_ptr(torch)
    want, want_norms = _clip_sgd_ref(theta0.cpu(), grad.cpu(), 0.01, 1.0)

    # a grid that can never be co-resident: the wait times out, the kernel drains, the error surfaces
    ctx.set_option("barrier_oversize", 2)
    ctx.set_option("barrier_timeout_us", 200000)
    th = theta0.clone()
    t0 = time.time()
    ctx.clip_sgd(st, th, grad, Z, 0.01, 1.0)
    with pytest.raises(_capi.SmamlError) as ei:
        ctx.sync(st)
    elapsed = time.time() - t0
    assert "grid-barrier" in str(ei.value) and "EHIP" in str(ei.value)
    assert elapsed < 30.0, elapsed
    ctx.sync(st)  # the flag was cleared with the report

    # back to the normal grid: correct results, fused and two-launch forms bitwise equal
    ctx.set_option("barrier_oversize", 0)
    ctx.set_option("barrier_timeout_us", 4000000)
    outs = []
    for fused in (1, 0):
        ctx.set_option("grid_barrier", fused)
        th = theta0.clone()
        norms = torch.empty(Z, device=DEV)
        ctx.clip_sgd(st, th, grad, Z, 0.01, 1.0, norms)
        ctx.sync(st)
        outs.append((th.cpu(), norms.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert rel(outs[0][0], want) < 1e-6
    np.testing.assert_allclose(outs[0][1].numpy(), want_norms, rtol=1e-6)
    ctx.close()


def test_grid_barrier_two_launch_form_bitwise_in_meta_step():
    """Second-order meta-step (k_inner_sgd every inner step, k_sweep_update every sweep step) with the
    fused grid-barrier launches and with the two-launch form: bitwise-equal losses, norms and
    meta-gradient."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=3, batch=2, order=2)
    P = synth.init_params(43, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(4300 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(2)]
    out = []
    for fused in (1, 0):
        ml = MetaLearner(d, cfg, Pg, Ptr, ei, device=DEV, task_group=None)
        ml.set_tasks(feats)
        ml.ctx.set_option("grid_barrier", fused)
        res = ml.meta_step()
        out.append((res.losses.cpu(), res.norms.cpu(), ml.meta_grad.cpu().clone()))
        del ml
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("cin", [8, 16])
def test_fused_gcn_few_input_channels(cin):
    """k_gcn_mlp at Hc = 256 with Cin0 <= 16: the layer-1 weight image has two zero-padded 16-k steps
    (the kernel always walks two), so layers 2..4 read their own images. Fused vs per-layer path and
    the oracle's GCN stack on every row."""
    d = ModelDims(num_nodes=441, input_channels=cin, output_channels=min(cin, 12))
    P = synth.init_params(51, d, gcn_bias_scale=0.1)
    _, Pg, _ = split(P)
    ei = grid_edges(d)
    ctx = _capi.Context(d, 0)
    ctx.set_graph(ei)
    ctx.set_gcn_params(params.pack({k: torch.from_numpy(v) for k, v in Pg.items()}, d, which=1, device=DEV))
    rng = np.random.default_rng(cin)
    xs_np = [rng.standard_normal((d.window_size * d.num_nodes, cin), dtype=np.float32) for _ in range(2)]
    xs = [torch.from_numpy(x).to(DEV) for x in xs_np]
    st = _capi.stream_ptr(torch)
    out = []
    for fused in (1, 0):
        ctx.set_option("gcn_fused", fused)
        F = torch.empty(len(xs), d.window_size * d.num_nodes, d.hidden_channels, device=DEV)
        ctx.gcn_forward(st, xs, F)
        ctx.sync(st)
        out.append(F.cpu().numpy())
    assert rel(out[0], out[1]) < 2e-6
    PT = refcpu.to_torch(P)
    Pgt = {k: v for k, v in PT.items() if k.startswith("base_stgcn")}
    for i, x in enumerate(xs_np):
        ref = refcpu.stgcn_features(torch.from_numpy(x), torch.from_numpy(ei).long(), Pgt).numpy()
        assert rel(out[0][i], ref) < 1e-5
    ctx.close()
