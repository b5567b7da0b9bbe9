"""f32 accuracy of the HIP path against a float64 restatement.

Every contraction on the hot path runs as f32-accurate products on the bf16 MFMA pipe
(gemm_core.h ``SMAML_X6``: each f32 operand split into three bf16 pieces, the six leading
piece products accumulated in f32) or, in the ``SMAML_X6=0`` build, on
``v_mfma_f32_32x32x2_f32``. Either way the claim is f32 arithmetic, so the test prices the GPU
result's error against float64 (the oracle run in f64 on the same inputs) next to the error of
the reference's own precision (the oracle in f32 on the CPU, MKL) and requires the GPU to be no
less accurate than that, up to a small factor for summation-order noise.

Workloads: BASELINE config-2 shapes (N=441, Hc=256, LSTM 4x128), one task, B=2, K=5 inner steps
(the bench's depth: the error of five chained Hessian-vector steps), second order, clip active and
inactive; and config-5 shapes (N=1024, Hc=512) at K=10 (ten chained steps): forward, BPTT, weight
gradients, the tangent sweep.

Special values (``test_bf16x6_special_values``): the split differs from an f32 MFMA only outside
the finite bf16 range. An inf operand gives NaN, not inf (x1 = x - x0 = inf - inf), and a finite
|x| >= 3.3961e38 (where RNE to bf16 overflows piece x0) gives NaN where f32 could still be finite;
every |x| below that is split exactly. Both cases stay non-finite, so a NaN/inf check downstream
sees them either way.
"""
import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import params, synth
from weatherforecast_stgcn_maml_amd.config import CONFIG2, CONFIG5, MamlConfig
from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph
from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
FACTOR = 3.0  # GPU error vs f64 may be at most this times the CPU-f32 error vs f64 (+ a floor)


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("d,K,B,max_norm,seed", [(CONFIG2, 5, 2, 1.0, 21), (CONFIG2, 5, 2, 0.02, 21),
                                                  (CONFIG5, 10, 1, 1.0, 27)],
                         ids=["cfg2-k5-clip1", "cfg2-k5-clip0.02", "cfg5-k10-clip1"])
def test_f32_accuracy_against_float64(d, K, B, max_norm, seed):
    """cfg5-k10: BASELINE config-5 shapes (N=1024, Hc=512, LSTM 4x128) at config 5's depth, ten chained
    Hessian-vector steps (the oracle takes ~1 min in f32 and ~2 min in f64 on the host)."""
    cfg = MamlConfig(inner_steps=K, batch=B, order=2, max_norm=max_norm)
    P = synth.init_params(seed, d, gcn_bias_scale=0.1)
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    theta = {k: P[k] for k in names}
    gcn = {k: v for k, v in P.items() if k not in names}
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(1300 if d is CONFIG2 else 1300 + seed, d.num_nodes, stream_len_for(cfg, d))
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml.set_tasks([feats])
    fast = torch.zeros(1, ml.theta.numel(), device=DEV)
    res = ml.meta_step(fast_out=fast)
    torch.cuda.synchronize()
    q = list(ml.default_windows()[-1, 0])
    S = cfg.inner_steps * cfg.batch

    def oracle(dtype):
        PT = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dtype) for k, v in P.items()}
        task = refcpu.TaskData(feats.astype(np.float64 if dtype == torch.float64 else np.float32), ei, d)
        return refcpu.meta_step({k: PT[k] for k in names}, {k: v for k, v in PT.items() if k not in names},
                                [task], q, cfg.inner_steps, cfg.batch, S, cfg.inner_lr, cfg.max_norm, 2)

    r64, r32 = oracle(torch.float64), oracle(torch.float32)
    mg = params.unpack(ml.meta_grad, d, 0)
    ad = params.unpack(fast[0], d, 0)
    rows = []
    for k in names:
        e_gpu = rel(mg[k].cpu().numpy(), r64["meta_grad"][k].numpy())
        e_cpu = rel(r32["meta_grad"][k].numpy(), r64["meta_grad"][k].numpy())
        rows.append(("meta_grad/" + k, e_gpu, e_cpu))
        e_gpu = rel(ad[k].cpu().numpy(), r64["adapted"][0][k].numpy())
        e_cpu = rel(r32["adapted"][0][k].numpy(), r64["adapted"][0][k].numpy())
        rows.append(("adapted/" + k, e_gpu, e_cpu))
    ql = float(res.losses.cpu().numpy()[-1, 0])
    rows.append(("query_mse", abs(ql - r64["query_losses"][0]) / r64["query_losses"][0],
                 abs(r32["query_losses"][0] - r64["query_losses"][0]) / r64["query_losses"][0]))
    worst = max(rows, key=lambda r: r[1] / max(r[2], 1e-7))
    print(f"\nN={d.num_nodes} K={K} max_norm={max_norm}: worst GPU/CPU-f32 error ratio {worst[0]}: gpu {worst[1]:.3e} cpu {worst[2]:.3e}; "
          f"mean gpu {np.mean([r[1] for r in rows]):.3e} cpu {np.mean([r[2] for r in rows]):.3e}")
    for name, e_gpu, e_cpu in rows:
        assert e_gpu <= FACTOR * e_cpu + 1e-7, (name, e_gpu, e_cpu)


def test_bf16x6_special_values():
    """The GCN drop-in (k_gcn_layer, staged bf16x6 split) on rows past the graph's nodes (self loop
    only, F3): finite inputs up to 3.38e38 are f32-accurate; inf and |x| in (3.3961e38, FLT_MAX]
    come out non-finite (NaN) on exactly the rows that hold them."""
    from weatherforecast_stgcn_maml_amd.model import GCNConv

    torch.manual_seed(3)
    d = CONFIG2
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    ei = torch.from_numpy(build_spatial_graph(lats, lons, 4)[0])
    conv = GCNConv(24, 64)
    with torch.no_grad():
        conv.lin.weight.mul_(1e-3)
    rows = d.num_nodes + 64
    x = torch.randn(rows, 24)
    big, inf, over = d.num_nodes + 3, d.num_nodes + 10, d.num_nodes + 20
    x[big, 5] = 3.38e38
    x[inf, 7] = float("inf")
    x[over, 2] = 3.40e38
    with torch.no_grad():
        out = conv.to(DEV)(x.to(DEV), ei.to(DEV)).cpu()
    ref = refcpu.gcn_conv(x.double(), ei, conv.lin.weight.detach().cpu().double(), conv.bias.detach().cpu().double())
    fin = [r for r in range(rows) if r not in (big, inf, over)]
    assert torch.isfinite(out[fin]).all() and torch.isfinite(out[big]).all()
    assert rel(out[fin].numpy(), ref[fin].numpy()) < 1e-6
    assert rel(out[big].numpy(), ref[big].numpy()) < 1e-6
    assert not torch.isfinite(out[inf]).any() and not torch.isfinite(out[over]).any()
