"""GPU parity of the finer-grained C ABI and of the torch.autograd shim
(§8(f) rank 2) against the CPU oracle (torch autograd through oracle/refcpu.py).

Tolerances (fp32): predictions, losses, parameters after training steps <= 1e-5 rel-L2
(SURVEY §8c); gradients <= 1e-4 rel-L2 (BPTT sums over T*N*B rows in a different order).
"""
import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import _capi, params, synth
from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2, MamlConfig
from weatherforecast_stgcn_maml_amd.maml import window_table

from test_gpu_parity import DEV, build_hybrid, grid_edges, rel, split

pytestmark = pytest.mark.gpu


def oracle_grads(P, x, y, ei, d):
    """loss and d loss / d (LSTM, head) of one sample through the oracle (CPU autograd)."""
    Pt = {k: torch.from_numpy(v).clone().requires_grad_(k.startswith(("lstm.", "output_layer.")))
          for k, v in P.items()}
    pred = refcpu.hybrid_forward(Pt, torch.from_numpy(x), torch.from_numpy(ei).long(), d)
    loss = refcpu.mse(pred, torch.from_numpy(y))
    loss.backward()
    return float(loss), pred.detach().numpy(), {k: v.grad.numpy() for k, v in Pt.items() if v.grad is not None}


@pytest.mark.parametrize("d", [CONFIG1, CONFIG2])
def test_autograd_shim_grads_match_oracle(d):
    P = synth.init_params(7, d, gcn_bias_scale=0.1)
    ei = grid_edges(d)
    feats = synth.make_features(synth.task_seed(3), d.num_nodes, synth.t_total_for(4))
    x, y = synth.sample_xy(feats, 2)
    loss_o, pred_o, g_o = oracle_grads(P, x, y, ei, d)

    m = build_hybrid(d, P).train()
    xg = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    pred = m(xg, torch.from_numpy(ei).to(DEV))
    assert pred.grad_fn is not None
    loss = torch.nn.functional.mse_loss(pred, torch.from_numpy(y).to(DEV))
    loss.backward()
    assert rel(pred.detach().cpu(), pred_o) < 1e-5
    assert abs(float(loss) - loss_o) < 1e-5 * loss_o
    sd = dict(m.named_parameters())
    for k, g in g_o.items():
        assert sd[k].grad is not None, k
        assert rel(sd[k].grad.cpu(), g) < 1e-4, (k, rel(sd[k].grad.cpu(), g))
    for k in sd:  # the reference runs the GCN under no_grad (F2)
        if k.startswith("base_stgcn."):
            assert sd[k].grad is None


def test_unmodified_sgd_loop_matches_oracle():
    """The reference's inner loop body (train_hybrid_maml_v5.py:130-139) written with plain
    torch calls -- loss.backward(), clip_grad_norm_, optim.SGD -- over the HIP module."""
    d = CONFIG1
    P = synth.init_params(11, d, gcn_bias_scale=0.1)
    ei = grid_edges(d)
    feats = synth.make_features(synth.task_seed(0), d.num_nodes, synth.t_total_for(6))

    def run(model_params, forward, steps=6):
        opt = torch.optim.SGD(model_params, lr=0.01)
        losses = []
        for i in range(steps):
            x, y = synth.sample_xy(feats, i)
            pred, yt = forward(x, y)
            loss = torch.nn.functional.mse_loss(pred, yt)
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model_params, 1.0)
            opt.step()
            losses.append(float(loss))
        return losses

    m = build_hybrid(d, P).train()
    eig = torch.from_numpy(ei).to(DEV)
    hip_losses = run(m.get_trainable_parameters(),
                     lambda x, y: (m(torch.from_numpy(np.ascontiguousarray(x)).to(DEV), eig),
                                   torch.from_numpy(y).to(DEV)))

    Pt = {k: torch.from_numpy(v).clone().requires_grad_(k.startswith(("lstm.", "output_layer.")))
          for k, v in P.items()}
    tr = [v for k, v in Pt.items() if v.requires_grad]
    eic = torch.from_numpy(ei).long()
    ora_losses = run(tr, lambda x, y: (refcpu.hybrid_forward(Pt, torch.from_numpy(x), eic, d), torch.from_numpy(y)))
    assert np.allclose(hip_losses, ora_losses, rtol=1e-5, atol=0)
    sd = dict(m.named_parameters())
    for k, v in Pt.items():
        if v.requires_grad:
            assert rel(sd[k].detach().cpu(), v.detach()) < 1e-5, k


def test_lstm_and_head_operators_match_oracle():
    d = CONFIG2
    P = synth.init_params(5, d, gcn_bias_scale=0.1)
    Ptr, Pg, names = split(P)
    ei = grid_edges(d)
    feats = synth.make_features(synth.task_seed(1), d.num_nodes, synth.t_total_for(3))
    xs, ys = zip(*[synth.sample_xy(feats, i) for i in range(2)])
    B, N, T, H = 2, d.num_nodes, d.window_size, d.lstm_hidden_size

    ctx = _capi.Context(d, 0)
    ctx.set_graph(ei)
    ctx.set_gcn_params(params.pack({k: torch.from_numpy(v) for k, v in Pg.items()}, d, which=1, device=DEV))
    theta = params.pack({k: torch.from_numpy(v) for k, v in Ptr.items()}, d, device=DEV)
    st = _capi.stream_ptr(torch)
    xg = [torch.from_numpy(np.ascontiguousarray(x)).to(DEV) for x in xs]
    yg = [torch.from_numpy(np.ascontiguousarray(y)).to(DEV) for y in ys]
    F = torch.empty(B, T * N, d.hidden_channels, device=DEV)
    ctx.gcn_forward(st, xg, F)
    hT = torch.empty(B, N, H, device=DEV)
    ctx.lstm_forward(st, theta, F, hT)
    pred = torch.empty(B, N * d.forecast_horizon, d.output_channels, device=DEV)
    loss = torch.empty(1, device=DEV)
    dpred = torch.empty_like(pred)
    ctx.head_loss(st, theta, hT, pred, yg, loss, dpred)
    Wo = params.unpack(theta, d)["output_layer.weight"]
    dhT = (dpred.view(B * N, -1) @ Wo).view(B, N, H).contiguous()
    grad = torch.empty_like(theta)
    ctx.lstm_backward(st, theta, dhT, grad)
    torch.cuda.synchronize()

    # oracle: per-sample MSE averaged over the batch (F9), autograd on CPU
    Pt = {k: torch.from_numpy(v).clone().requires_grad_(k in names) for k, v in P.items()}
    eic = torch.from_numpy(ei).long()
    Fo = [refcpu.stgcn_features(torch.from_numpy(x), eic, Pt).detach() for x in xs]
    seq = torch.cat([f.view(T, N, -1).permute(1, 0, 2) for f in Fo])
    hTo = refcpu.lstm_stack(seq, Pt, d.lstm_num_layers)
    predo = (hTo @ Pt["output_layer.weight"].t() + Pt["output_layer.bias"]).view(B, N * d.forecast_horizon, -1)
    losso = torch.stack([refcpu.mse(predo[b], torch.from_numpy(ys[b])) for b in range(B)]).mean()
    losso.backward()

    assert rel(F.cpu(), torch.stack(Fo)) < 1e-5
    assert rel(hT.cpu(), hTo.detach().view(B, N, H)) < 1e-5
    assert rel(pred.cpu(), predo.detach()) < 1e-5
    assert abs(float(loss) - float(losso)) < 1e-5 * float(losso)
    g = params.unpack(grad, d)
    for k in names:
        if k.startswith("lstm."):
            assert rel(g[k].cpu(), Pt[k].grad) < 1e-4, k
        else:
            assert float(g[k].abs().max()) == 0.0, k  # lstm_backward leaves the head to the caller
    # prediction-only head
    pred2 = torch.empty_like(pred)
    ctx.head_loss(st, theta, hT, pred2)
    torch.cuda.synchronize()
    assert torch.equal(pred2, pred)


def test_backward_requires_forward_and_is_consumed():
    d = CONFIG1
    P = synth.init_params(2, d)
    Ptr, Pg, _ = split(P)
    ctx = _capi.Context(d, 0)
    ctx.set_graph(grid_edges(d))
    ctx.set_gcn_params(params.pack({k: torch.from_numpy(v) for k, v in Pg.items()}, d, which=1, device=DEV))
    theta = params.pack({k: torch.from_numpy(v) for k, v in Ptr.items()}, d, device=DEV)
    grad = torch.empty_like(theta)
    dpred = torch.zeros(d.num_nodes * d.forecast_horizon, d.output_channels, device=DEV)
    st = _capi.stream_ptr(torch)
    with pytest.raises(_capi.SmamlError, match="ESTATE"):
        ctx.backward(st, theta, dpred, grad)
    feats = synth.make_features(synth.task_seed(0), d.num_nodes, synth.t_total_for(1))
    x, _ = synth.sample_xy(feats, 0)
    pred = torch.empty_like(dpred)
    ctx.forward(st, theta, [torch.from_numpy(np.ascontiguousarray(x)).to(DEV)], pred)
    ctx.backward(st, theta, dpred, grad)
    torch.cuda.synchronize()
    assert float(grad.abs().max()) == 0.0  # zero upstream gradient
    with pytest.raises(_capi.SmamlError, match="ESTATE"):  # activations consumed (dG in place)
        ctx.backward(st, theta, dpred, grad)


def test_clip_sgd_matches_torch():
    d = CONFIG2
    ctx = _capi.Context(d, 0)
    P = params.trainable_layout(d)[1]
    g = torch.Generator().manual_seed(0)
    theta = torch.randn(3, P, generator=g).to(DEV)
    grad = (torch.randn(3, P, generator=g) * torch.tensor([[0.001], [1.0], [30.0]])).to(DEV)
    norms = torch.empty(3, device=DEV)
    ref = theta.clone()
    for z in range(3):
        n = float(grad[z].double().norm())
        coef = min(1.0 / (n + 1e-6), 1.0)
        ref[z] -= 0.01 * grad[z] * coef
    ctx.clip_sgd(_capi.stream_ptr(torch), theta, grad, 3, 0.01, 1.0, norms)
    torch.cuda.synchronize()
    assert rel(theta.cpu(), ref.cpu()) < 1e-6
    assert np.allclose(norms.cpu().numpy(), grad.double().norm(dim=1).cpu().numpy(), rtol=1e-5)


def test_inner_loop_equals_meta_step_fast_weights():
    d = CONFIG1
    P = synth.init_params(3, d)
    Ptr, Pg, _ = split(P)
    ctx = _capi.Context(d, 0)
    ctx.set_graph(grid_edges(d))
    ctx.set_gcn_params(params.pack({k: torch.from_numpy(v) for k, v in Pg.items()}, d, which=1, device=DEV))
    theta = params.pack({k: torch.from_numpy(v) for k, v in Ptr.items()}, d, device=DEV)
    streams = [torch.from_numpy(synth.make_features(synth.task_seed(j), d.num_nodes, synth.t_total_for(8))).to(DEV)
               for j in range(2)]
    ctx.set_tasks(streams)
    K, B = 3, 2
    w = window_table(MamlConfig(inner_steps=K, batch=B), 2)
    st = _capi.stream_ptr(torch)
    fa = torch.empty(2, theta.numel(), device=DEV)
    fb = torch.empty_like(fa)
    la = torch.empty(K + 1, 2, device=DEV)
    lb = torch.empty_like(la)
    ctx.inner_loop(st, theta, K, B, w, 0.01, 1.0, fa, la)
    ctx.meta_step(st, theta, 0, K, B, w, 0.01, 1.0, 1.0, losses=lb, fast_out=fb)
    torch.cuda.synchronize()
    assert torch.equal(fa, fb) and torch.equal(la, lb)


def test_alloc_free_and_world1_comm():
    d = CONFIG1
    ctx = _capi.Context(d, 0)
    p = ctx.alloc(1 << 20)
    assert p
    ctx.free(p)
    uid = _capi.comm_unique_id()
    assert len(uid) == 128
    ctx.comm_init(0, 1, uid)
    buf = torch.arange(1000, dtype=torch.float32, device=DEV)
    ref = buf.clone()
    ctx.comm_allreduce(_capi.stream_ptr(torch), buf)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)  # world 1: sum over one rank
    ctx.comm_destroy()


# ----------------------------------------------------------------------------- module-API dropout
def _module(d, P, p_gcn, p_lstm):
    from weatherforecast_stgcn_maml_amd.hybrid_model import HybridSTGCN_LSTM
    from weatherforecast_stgcn_maml_amd.model import STGCN

    base = STGCN(d.input_channels, d.hidden_channels, d.output_channels, d.window_size, d.forecast_horizon,
                 dropout_rate=p_gcn)
    m = HybridSTGCN_LSTM(base, d.lstm_hidden_size, d.lstm_num_layers, p_lstm, d.output_channels,
                         d.forecast_horizon, freeze_base=True)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    return m.to("cuda:0")


@pytest.mark.parametrize("d", [CONFIG1, CONFIG2])
def test_train_mode_module_dropout_matches_oracle(d):
    """HybridSTGCN_LSTM in train() mode with the reference's dropout sites (STGCN dropout after
    conv1-3, hybrid_model.py:67,70,73; nn.LSTM inter-layer dropout :42-49; head input :108):
    an unmodified loss.backward() through the autograd shim reproduces the oracle's loss and
    gradients under the same counter-based masks (seed drawn from the torch RNG per call)."""
    from weatherforecast_stgcn_maml_amd.hybrid_model import draw_dropout_seed

    P = synth.init_params(41, d, gcn_bias_scale=0.1)
    m = _module(d, P, 0.2, 0.2).train()
    ei = grid_edges(d)
    feats = synth.make_features(4400, d.num_nodes, synth.t_total_for(2))
    x, y = synth.sample_xy(feats, 1)
    xg = torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")
    yg = torch.from_numpy(np.ascontiguousarray(y)).to("cuda:0")
    torch.manual_seed(77)
    pred = m(xg, torch.from_numpy(ei).to("cuda:0"))
    loss = torch.nn.MSELoss()(pred, yg)
    loss.backward()
    torch.manual_seed(77)
    seed = draw_dropout_seed()
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    PT = refcpu.to_torch(P)
    Pt = {k: PT[k].clone().requires_grad_(True) for k in names}
    task = refcpu.TaskData(feats, ei, d)
    ref_loss, ref_pred = refcpu.batch_loss(Pt, {k: v for k, v in PT.items() if k not in names}, task, [1],
                                           refcpu.Dropout(seed, 0.2, 0.2, 0, 0))
    ref_loss.backward()
    assert rel(pred.detach().cpu().numpy(), ref_pred[0].detach().numpy()) < 1e-5
    assert abs(float(loss) - float(ref_loss)) < 1e-5 * float(ref_loss)
    got = {"lstm." + n: p.grad for n, p in m.lstm.named_parameters()}
    got["output_layer.weight"] = m.output_layer.weight.grad
    got["output_layer.bias"] = m.output_layer.bias.grad
    for k in names:
        assert rel(got[k].cpu().numpy(), Pt[k].grad.numpy()) < 1e-4, k
    # eval() and a second train-mode call: no dropout / fresh masks
    m.eval()
    with torch.no_grad():
        p_eval = m(xg, torch.from_numpy(ei).to("cuda:0"))
        p_eval2 = m(xg, torch.from_numpy(ei).to("cuda:0"))
    assert torch.equal(p_eval, p_eval2)
    m.train()
    with torch.no_grad():
        p2 = m(xg, torch.from_numpy(ei).to("cuda:0"))
    assert not torch.equal(p2, pred.detach()) and not torch.equal(p2, p_eval)


@pytest.mark.parametrize("i", [0, 1])
def test_stgcn_forward_matches_reference(golden_dir, i):
    """The drop-in model.STGCN.forward (model.py:30-52: conv x4 + ReLU, last time block,
    output_layer, view/reshape) against the reference module's own output (eval mode), and in
    train mode (dropout after each of the four convs) against the oracle's masks."""
    import os
    from weatherforecast_stgcn_maml_amd.hybrid_model import draw_dropout_seed
    from weatherforecast_stgcn_maml_amd.model import STGCN

    z = np.load(os.path.join(golden_dir, "stgcn_forward.npz"))
    d = CONFIG1 if int(z[f"d{i}/num_nodes"]) == CONFIG1.num_nodes else CONFIG2
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    base = STGCN(d.input_channels, d.hidden_channels, d.output_channels, d.window_size, d.forecast_horizon,
                 dropout_rate=0.2)
    base.load_state_dict({k[len("base_stgcn."):]: torch.from_numpy(v) for k, v in P.items()
                          if k.startswith("base_stgcn.")})
    base = base.to("cuda:0").eval()
    x, _ = synth.sample_xy(synth.make_features(int(z["feat_seed"]), d.num_nodes, synth.t_total_for(1)), 0)
    xg = torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")
    eig = torch.from_numpy(z[f"d{i}/edge_index"]).to("cuda:0")
    out = base(xg, eig).detach().cpu().numpy()
    assert out.shape == z[f"d{i}/out"].shape
    assert rel(out, z[f"d{i}/out"]) < 1e-5
    base.train()
    torch.manual_seed(3)
    out_t = base(xg, eig).detach().cpu()
    torch.manual_seed(3)
    drop = refcpu.Dropout(draw_dropout_seed(), 0.2, 0.0, 0, 0)
    ref = refcpu.stgcn_forward(torch.from_numpy(np.ascontiguousarray(x)), torch.from_numpy(z[f"d{i}/edge_index"]),
                               refcpu.to_torch(P), d, drop)
    assert rel(out_t.numpy(), ref.numpy()) < 1e-5
    assert rel(out_t.numpy(), out) > 1e-3


@pytest.mark.parametrize("name", ["cfg1_validate.npz", "cfg2_validate.npz"])
def test_evaluate_regional_matches_validate_adapted(golden_dir, name):
    """evaluate.evaluate_regional (HIP forward of the first 3 windows, sample / node means on
    the device, denormalised per-variable MSE / MAE) against validate_hybrid_v5.validateAdapted
    run unmodified on the same synthetic stream (tests/golden/cfg*_validate.npz)."""
    import os
    from weatherforecast_stgcn_maml_amd.evaluate import evaluate_regional

    z = np.load(os.path.join(golden_dir, name))
    d = CONFIG1 if name.startswith("cfg1") else CONFIG2
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    m = _module(d, P, 0.2, 0.2).eval()
    feats = torch.from_numpy(synth.make_features(int(z["feat_seed"]), d.num_nodes, int(z["t_sub"]))).to("cuda:0")
    res = evaluate_regional(m, feats, grid_edges(d), {"mean": z["stats_mean"], "std": z["stats_std"]})
    for v in z["var_names"]:
        v = str(v)
        for k in ("mse", "mae"):
            want = float(z[f"{v}/{k}"])
            assert abs(res[v][k] - want) <= 1e-4 * abs(want), (v, k, res[v][k], want)
    assert abs(res["average_mse"] - float(z["average_mse"])) <= 1e-4 * float(z["average_mse"])


@pytest.mark.parametrize("p_gcn", [0.0, 0.2])
def test_fused_gcn_matches_per_layer(p_gcn):
    """The fused GCN stack (k_gcn_mlp: rows t >= 1, all four convs in registers) and the t = 0 rows'
    per-layer path against the all-rows per-layer kernel (gcn_fused 0): same features and
    predictions up to summation order, the same dropout masks (conv1..conv3 at p_gcn), and at
    p_gcn = 0 the oracle's GCN stack (hybrid_model.py:60-78) on every row."""
    d = CONFIG2
    P = synth.init_params(33, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    ctx = _capi.Context(d, 0)
    ctx.set_graph(ei)
    ctx.set_gcn_params(params.pack({k: torch.from_numpy(v) for k, v in Pg.items()}, d, which=1, device=DEV))
    theta = params.pack({k: torch.from_numpy(v) for k, v in Ptr.items()}, d, device=DEV)
    feats = synth.make_features(synth.task_seed(3), d.num_nodes, synth.t_total_for(8))
    xs_np = [np.ascontiguousarray(synth.sample_xy(feats, i)[0]) for i in (0, 3, 7)]
    xs = [torch.from_numpy(x).to(DEV) for x in xs_np]
    st = _capi.stream_ptr(torch)
    ctx.set_task_ids([5])
    out = []
    for fused in (1, 0):
        ctx.set_option("gcn_fused", fused)
        ctx.set_dropout(p_gcn, 0.0, 77)
        pred = torch.empty(len(xs) * d.num_nodes * d.forecast_horizon, d.output_channels, device=DEV)
        F = torch.empty(len(xs), d.window_size * d.num_nodes, d.hidden_channels, device=DEV)
        ctx.forward(st, theta, xs, pred, F)
        torch.cuda.synchronize()
        out.append((F.cpu().numpy(), pred.cpu().numpy()))
    (Ff, pf), (Fl, pl) = out
    assert rel(Ff, Fl) < 2e-6 and rel(pf, pl) < 2e-6
    # identical dropout masks: the zero patterns (dropout and ReLU) agree up to ReLU ties at rounding level
    assert np.mean((Ff == 0) != (Fl == 0)) < 1e-5
    if p_gcn == 0.0:
        PT = refcpu.to_torch(P)
        Pgt = {k: v for k, v in PT.items() if k.startswith("base_stgcn")}
        for i, x in enumerate(xs_np):
            ref = refcpu.stgcn_features(torch.from_numpy(x), torch.from_numpy(ei).long(), Pgt).numpy()
            assert rel(Ff[i], ref) < 1e-5


def test_gate_images_bitwise():
    """The gate GEMMs fed from pre-split weight images (launch_split_gate: bf16 pieces copied into
    LDS with direct-to-LDS loads) form the same products as splitting the f32 weights in every
    workgroup, in the same order: the meta-step's losses and meta-gradient are bitwise equal."""
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=2, order=2)
    P = synth.init_params(37, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(3700 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(2)]
    out = []
    for img in (1, 0):
        ml = MetaLearner(d, cfg, Pg, Ptr, ei, device=DEV, task_group=None)
        ml.set_tasks(feats)
        ml.ctx.set_option("gate_img", img)
        ml.ctx.variant_counts(reset=True)
        res = ml.meta_step()
        vc = ml.ctx.variant_counts()
        assert (vc["fwd_img"] > 0) == bool(img), vc
        out.append((res.losses.cpu(), ml.meta_grad.cpu().clone()))
        del ml
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("knob", ["wgrad_wide", "wgrad_pair"])
def test_wgrad_variants_match(knob):
    """wgrad_wide: weight
    gradients with 256-column problems (LSTM layers >= 1 and their tangent passes) on 256 x 256 tiles
    (kernels.hip CfgTW); the 512 x 128 tiles give the same weight sums (same split-K slices, same
    per-element MFMA order) and the bias column sums up to summation order. wgrad_pair: the tangent
    weight gradient's two passes (R(dG)^T [x|h] and dG^T [Rx|Rh]) as one split-K launch instead of two
    accumulating ones (summation order only). Both second-order meta-steps agree with each other well
    inside the oracle tolerance."""
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=2, order=2)
    P = synth.init_params(41, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(4100 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(2)]
    out = []
    for on in (1, 0):
        ml = MetaLearner(d, cfg, Pg, Ptr, ei, device=DEV, task_group=None)
        ml.set_tasks(feats)
        ml.ctx.set_option(knob, on)
        ml.ctx.variant_counts(reset=True)
        res = ml.meta_step()
        vc = ml.ctx.variant_counts()
        assert vc["wgrad"] > 0 and (vc[knob] > 0) == bool(on), vc
        out.append((res.losses.cpu().numpy(), ml.meta_grad.cpu().numpy().copy()))
        del ml
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=1e-6)
    assert rel(out[0][1], out[1][1]) < 1e-6


@pytest.mark.parametrize("d", [CONFIG1, CONFIG2], ids=["cfg1", "cfg2"])
@pytest.mark.parametrize("p", [0.0, 0.2])
def test_stgcn_autograd_matches_oracle(d, p):
    """STGCN trained on its own (model.py:30-52 as an ordinary differentiable module): the HIP path's
    forward and backward (_STGCNFn: conv + ReLU x4 with train-mode dropout, the head; backward through
    smaml_gcn_conv_backward / smaml_relu_mask / the replayed masks) against torch autograd through the
    oracle's STGCN (refcpu.stgcn_forward, PyG gcn_norm restated) with the same masks: loss, the output,
    the gradient of every parameter and of the input x."""
    from weatherforecast_stgcn_maml_amd.hybrid_model import draw_dropout_seed
    from weatherforecast_stgcn_maml_amd.model import STGCN

    P = synth.init_params(53, d, gcn_bias_scale=0.1)
    base = STGCN(d.input_channels, d.hidden_channels, d.output_channels, d.window_size, d.forecast_horizon,
                 dropout_rate=p)
    base.load_state_dict({k[len("base_stgcn."):]: torch.from_numpy(v) for k, v in P.items()
                          if k.startswith("base_stgcn.")})
    base = base.to(DEV).train()
    x, _ = synth.sample_xy(synth.make_features(5300, d.num_nodes, synth.t_total_for(1)), 0)
    ei = grid_edges(d)
    rng = np.random.default_rng(7)
    R = rng.standard_normal((d.num_nodes * d.forecast_horizon, d.output_channels)).astype(np.float32)
    xg = torch.from_numpy(np.ascontiguousarray(x)).to(DEV).requires_grad_(True)
    torch.manual_seed(11)
    out = base(xg, torch.from_numpy(ei).to(DEV))
    assert out.grad_fn is not None
    (out * torch.from_numpy(R).to(DEV)).sum().backward()
    # oracle: the same masks (the module draws its seed from torch's RNG)
    torch.manual_seed(11)
    drop = refcpu.Dropout(draw_dropout_seed(), p, 0.0, 0, 0) if p > 0.0 else None
    Pt = {k: v.clone().requires_grad_(True) for k, v in refcpu.to_torch(P).items() if k.startswith("base_stgcn.")}
    xt = torch.from_numpy(np.ascontiguousarray(x)).clone().requires_grad_(True)
    ref = refcpu.stgcn_forward(xt, torch.from_numpy(ei).long(), Pt, d, drop)
    (ref * torch.from_numpy(R)).sum().backward()
    assert rel(out.detach().cpu(), ref.detach()) < 1e-5
    sd = dict(base.named_parameters())
    for k, v in Pt.items():
        g = sd[k[len("base_stgcn."):]].grad
        assert g is not None, k
        assert rel(g.cpu(), v.grad) < 1e-4, (k, rel(g.cpu(), v.grad))
    assert rel(xg.grad.cpu(), xt.grad) < 1e-4


@pytest.mark.parametrize("knob", ["bwdd_remap", "gcn_dedup", "gcn_dedup_layers", "bptt_streams", "fwd_streams",
                                  "f_compact", "f_compact_layers"])
def test_order_only_knobs_bitwise(knob):
    """Knobs that only reorder or deduplicate work (bwdd_remap: the tangent BPTT's pair-segment tile
    order per XCD; gcn_dedup: the fused GCN rows of consecutive windows once per distinct stream row,
    stored to every sample holding them; gcn_dedup_layers: the same on the per-layer GCN path,
    gcn_fused 0, as one pseudo-sample of distinct stream rows per task expanded into F; bptt_streams /
    fwd_streams: every BPTT / forward diagonal in two row chunks on side streams, always on the big tiles,
    the weight gradients after the sweep; f_compact: the features of those steps stored once per distinct
    stream row, read only through the layer-0 projection tables and the gathered dW_ih0 -- fused and per-layer
    GCN paths, 2 tasks x B = 8 so every layer-0 diagonal runs the big tiles) leave every
    row's arithmetic unchanged: a second-order meta-step (big tangent BPTT tiles forced, every primal
    kept) is bitwise equal with the knob on and off."""
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    d = CONFIG2
    compact = knob.startswith("f_compact")
    cfg = MamlConfig(inner_steps=2, batch=8 if compact else 4, order=2)
    P = synth.init_params(47, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(4700 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(2 if compact else 3)]
    out = []
    for on in (1, 0):
        ml = MetaLearner(d, cfg, Pg, Ptr, ei, device=DEV, task_group=None)
        ml.set_tasks(feats)
        ml.ctx.set_option("bwdd_big_min", 0)
        if knob.endswith("_layers"):
            ml.ctx.set_option("gcn_fused", 0)
        if knob.endswith("_streams"):
            ml.ctx.set_option("bwd_big_min", 0)  # (chunked diagonals always run the big tiles: both arms do)
            ml.ctx.set_option(knob, 2 if on else 1)
        else:
            ml.ctx.set_option(knob.removesuffix("_layers"), on)
        ml.ctx.variant_counts(reset=True)
        res = ml.meta_step()
        vc = ml.ctx.variant_counts()
        assert vc["bwd_dual_big_kept"] > 0, vc
        if knob.startswith("gcn_dedup"):
            assert (vc["gcn_dedup"] > 0) == bool(on), vc
        if knob.startswith("f_compact"):  # every step: K inner steps + the query; the sweep reads them from so_F
            assert vc["f_compact"] == (cfg.inner_steps + 1 if on else 0), vc
        out.append((res.losses.cpu(), res.norms.cpu(), ml.meta_grad.cpu().clone()))
        del ml
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def test_row_chunks_bitwise_cfg5_corner_diagonals():
    """The configuration that raced in round 5 (DESIGN.md "row chunks on side streams"): BASELINE config-5
    shapes (N = 1024, Hc = 512), ONE task, B = 12, so the 4-problem BPTT diagonals are big by the default
    tile threshold while the 1-problem corner diagonals are not -- with row chunks every chunked diagonal
    must still run the row-restricted big tiles, or a whole-row launch on one stream would race the other
    stream's chunk. Forward and BPTT chunks on (fwd_streams = bptt_streams = 2, default thresholds) against
    one stream with the big tiles forced everywhere: the K = 2 second-order meta-step is bitwise equal,
    and the launch counters show every diagonal, the corners included, on the big tiles
    (hybrid_model.py:93-102 / train_hybrid_maml_v5.py:134 through the wavefront)."""
    from weatherforecast_stgcn_maml_amd.config import CONFIG5
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    d = CONFIG5
    cfg = MamlConfig(inner_steps=2, batch=12, order=2)
    K, diags = cfg.inner_steps, d.window_size + d.lstm_num_layers - 1
    P = synth.init_params(61, d, gcn_bias_scale=0.1)
    Ptr, Pg, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(6100, d.num_nodes, stream_len_for(cfg, d))]
    out = []
    for chunks in (2, 1):
        ml = MetaLearner(d, cfg, Pg, Ptr, ei, device=DEV, task_group=1)
        ml.set_tasks(feats)
        ml.ctx.set_option("fwd_streams", chunks)
        ml.ctx.set_option("bptt_streams", chunks)
        if chunks == 1:  # (the one-stream arm on the big tiles everywhere, as every chunked diagonal runs)
            ml.ctx.set_option("bwd_big_min", 0)
            ml.ctx.set_option("bwdd_big_min", 0)
        ml.ctx.variant_counts(reset=True)
        ml.ctx.timing_collect()
        ml.ctx.timing(True)
        res = ml.meta_step()
        kern = ml.ctx.timing_collect()
        ml.ctx.timing(False)
        vc = ml.ctx.variant_counts()
        assert vc["bwd_big"] == (K + 1) * diags and vc["bwd_small"] == 0 and vc["bwd_split"] == 0, vc
        assert vc["bwd_dual_big_kept"] == K * diags and vc["bwd_dual_small_kept"] == 0, vc
        assert vc["fwd"] == (K + 1) * diags and vc["fwd_split"] == 0 and vc["fwd_kw"] == 0, vc
        walls = {k for k, v in kern.items() if k.endswith("_wall") and v["launches"] > 0}
        if chunks == 2:  # every sweep ran chunked: primal forward / BPTT, tangent forward / BPTT
            assert walls == {"lstm_fwd_step_wall", "lstm_bwd_step_wall", "lstm_fwd_dual_wall", "lstm_bwd_dual_wall"}, kern
        else:
            assert not walls, kern
        out.append((res.losses.cpu(), res.norms.cpu(), ml.meta_grad.cpu().clone()))
        del ml
        torch.cuda.empty_cache()
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
