"""GPU parity: the HIP path (through the C ABI) against the golden fixtures made by the
reference itself and against the CPU oracle.

Tolerances (fp32): query MSE <= 1e-4 rel (BASELINE); predictions, per-step
losses, adapted parameters <= 1e-5 rel-L2 (F11 makes the MSE alone a weak signal);
meta-gradients <= 1e-4 rel-L2.
"""
import os

import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import _capi, params, synth
from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2, CONFIG5, MamlConfig, ModelDims
from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph
from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for, window_table

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def split(P):
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    return {k: P[k] for k in names}, {k: v for k, v in P.items() if k not in names}, names


def grid_edges(d):
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    return build_spatial_graph(lats, lons, 4)[0]


def build_hybrid(d, P):
    from weatherforecast_stgcn_maml_amd.hybrid_model import HybridSTGCN_LSTM
    from weatherforecast_stgcn_maml_amd.model import STGCN

    base = STGCN(d.input_channels, d.hidden_channels, d.output_channels, d.window_size,
                 d.forecast_horizon, dropout_rate=0.0)
    m = HybridSTGCN_LSTM(base, d.lstm_hidden_size, d.lstm_num_layers, 0.0, d.output_channels,
                         d.forecast_horizon, freeze_base=False)
    assert list(m.state_dict().keys()) == list(P.keys())
    m.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    return m.to(DEV).eval()


# ----------------------------------------------------------------------------- forward
@pytest.mark.parametrize("d,name", [(CONFIG1, "cfg1_ref.npz"), (CONFIG2, "cfg2_ref.npz")])
def test_forward_matches_reference(golden_dir, d, name):
    z = load(golden_dir, name)
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    m = build_hybrid(d, P)
    feats = synth.make_features(int(z["feat_seeds"][0]), d.num_nodes, synth.t_total_for(int(z["n_samples"])))
    x, y = synth.sample_xy(feats, 0)
    xg = torch.from_numpy(np.ascontiguousarray(x)).to(DEV)
    eig = torch.from_numpy(z["edge_index"]).to(DEV)
    with torch.no_grad():  # eval-style call (the module is differentiable otherwise)
        pred = m(xg, eig).cpu().numpy()
    assert pred.shape == z["pred0"].shape
    assert rel(pred, z["pred0"]) < 1e-5
    mse = float(((pred - y) ** 2).mean())
    assert abs(mse - float(z["loss0"])) < 1e-5 * float(z["loss0"])
    f = m.extract_base_features(xg, eig).cpu().numpy()
    if "feats0" in z:
        assert rel(f, z["feats0"]) < 1e-5
    else:
        assert abs(f.astype(np.float64).sum() - float(z["feats0_sum"])) < 1e-5 * abs(float(z["feats0_sum"]))


def test_gcnconv_dropin_matches_oracle():
    """PyG GCNConv drop-in, forward and (round 4) backward, against the oracle's restatement run through
    torch autograd (the t = 0 block aggregates, later rows see only their self loop, F3)."""
    from weatherforecast_stgcn_maml_amd.model import GCNConv

    torch.manual_seed(0)
    d = CONFIG2
    ei = grid_edges(d)
    for cin, cout, rows in [(24, 256, 24 * 441), (256, 256, 3 * 441 + 17), (8, 64, 441)]:
        conv = GCNConv(cin, cout)
        with torch.no_grad():
            conv.bias.uniform_(-0.1, 0.1)
        x = torch.randn(rows, cin)
        W = conv.lin.weight.detach().clone().requires_grad_(True)
        b = conv.bias.detach().clone().requires_grad_(True)
        xr = x.clone().requires_grad_(True)
        ref = refcpu.gcn_conv(xr, torch.from_numpy(ei), W, b)
        R = torch.randn(rows, cout)
        (ref * R).sum().backward()
        conv = conv.to(DEV)
        xg = x.to(DEV).requires_grad_(True)
        out = conv(xg, torch.from_numpy(ei).to(DEV))
        assert rel(out.detach().cpu().numpy(), ref.detach().numpy()) < 1e-5
        # backward on the HIP path (smaml_gcn_conv_backward: A_hat^T dz W, dz^T A_hat x, sum dz)
        (out * R.to(DEV)).sum().backward()
        assert rel(conv.lin.weight.grad.cpu(), W.grad) < 1e-5
        assert rel(conv.bias.grad.cpu(), b.grad) < 1e-5
        assert rel(xg.grad.cpu(), xr.grad) < 1e-5


# ----------------------------------------------------------------------------- reference mode
def run_reference_mode(d, z, tasks, steps, support):
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    cfg = MamlConfig(inner_steps=steps, batch=1, order=0, support_samples=support)
    ml = MetaLearner(d, cfg, gcn, theta, z["edge_index"], device=DEV)
    feats = [synth.make_features(int(z["feat_seeds"][j]), d.num_nodes, synth.t_total_for(int(z["n_samples"])))
             for j in range(tasks)]
    ml.set_tasks(feats)
    fast = torch.zeros(tasks, ml.theta.numel(), device=DEV)
    theta0 = ml.theta.clone()
    res = ml.meta_step(fast_out=fast)
    assert torch.equal(theta0, ml.theta), "reference mode must leave theta unchanged (F1)"
    return res, fast, names


def test_reference_inner_loop_cfg1(golden_dir):
    """inner_loop_v4 with its real constants: 6 epochs x 15 support samples, batch 1."""
    d = CONFIG1
    z = load(golden_dir, "cfg1_ref.npz")
    steps = int(z["inner_epochs"]) * 15
    res, fast, names = run_reference_mode(d, z, 2, steps, int(z["n_support"]))
    losses = res.losses.cpu().numpy()
    norms = res.norms.cpu().numpy()
    for j in range(2):
        assert rel(losses[:steps, j], z[f"t{j}_losses"]) < 1e-5
        assert rel(norms[:, j], z[f"t{j}_norms"]) < 1e-5
        ad = params.unpack(fast[j], d, 0)
        for k in names:
            assert rel(ad[k].cpu().numpy(), z[f"t{j}_adapted/{k}"]) < 1e-5, k
        q = float(losses[steps, j])
        assert abs(q - float(z[f"t{j}_query_mse"])) < 1e-4 * float(z[f"t{j}_query_mse"])
    assert abs(res.meta_loss - float(z["meta_loss"])) < 1e-4 * float(z["meta_loss"])


def test_reference_inner_loop_cfg2(golden_dir):
    d = CONFIG2
    z = load(golden_dir, "cfg2_ref.npz")
    steps = int(z["inner_epochs"]) * int(z["n_support"])
    res, fast, names = run_reference_mode(d, z, 1, steps, int(z["n_support"]))
    losses = res.losses.cpu().numpy()
    assert rel(losses[:steps, 0], z["t0_losses"]) < 1e-5
    assert rel(res.norms.cpu().numpy()[:, 0], z["t0_norms"]) < 1e-5
    ad = params.unpack(fast[0], d, 0)
    for k in names:
        v = ad[k].cpu().numpy().astype(np.float64)
        assert abs(np.linalg.norm(v) - float(z[f"t0_adapted_norm/{k}"])) < 1e-5 * np.linalg.norm(v), k
        assert rel(v.reshape(-1)[:64], z[f"t0_adapted_slice/{k}"]) < 1e-5, k
    q = float(losses[steps, 0])
    assert abs(q - float(z["t0_query_mse"])) < 1e-4 * float(z["t0_query_mse"])


# ----------------------------------------------------------------------------- MAML (B > 1)
@pytest.mark.parametrize("clip", [0, 1])
def test_first_order_meta_grad_cfg1(golden_dir, clip):
    d = CONFIG1
    z = load(golden_dir, "cfg1_maml.npz")
    steps, batch, support, qb = (int(z[k]) for k in ("steps", "batch", "support", "qbatch"))
    assert qb == batch
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    cfg = MamlConfig(inner_steps=steps, batch=batch, order=1, support_samples=support,
                     max_norm=float(z["max_norms"][clip]))
    ml = MetaLearner(d, cfg, gcn, theta, z["edge_index"], device=DEV)
    feats = [synth.make_features(int(s), d.num_nodes, synth.t_total_for(support + qb)) for s in z["feat_seeds"]]
    ml.set_tasks(feats)
    fast = torch.zeros(len(feats), ml.theta.numel(), device=DEV)
    res = ml.meta_step(windows=window_table(cfg, len(feats)), fast_out=fast)
    losses = res.losses.cpu().numpy()
    total = {k: 0.0 for k in names}
    for j in range(len(feats)):
        tag = f"t{j}_c{clip}_o1"
        assert rel(losses[:steps, j], z[tag + "_losses"]) < 1e-5
        assert abs(losses[steps, j] - float(z[tag + "_query"])) < 1e-5 * float(z[tag + "_query"])
        ad = params.unpack(fast[j], d, 0)
        for k in names:
            assert rel(ad[k].cpu().numpy(), z[f"{tag}_adapted/{k}"]) < 1e-5, k
            total[k] = total[k] + z[f"{tag}_metagrad/{k}"]
    # meta_grad was consumed by AdamW but is kept in ml.meta_grad (summed over tasks)
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), total[k]) < 1e-4, k


def test_meta_step_matches_oracle_cfg2_batched():
    """Config-2 shapes with B=2, K=2, 2 tasks: losses, adapted params, FO meta-grad."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=2, order=1)
    P = synth.init_params(5, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    T = stream_len_for(cfg, d)
    feats = [synth.make_features(1000 + j, d.num_nodes, T) for j in range(2)]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml.set_tasks(feats)
    fast = torch.zeros(2, ml.theta.numel(), device=DEV)
    res = ml.meta_step(fast_out=fast)
    PT = refcpu.to_torch(P)
    Pg = {k: v for k, v in PT.items() if k not in names}
    S = cfg.inner_steps * cfg.batch
    tasks = [refcpu.TaskData(f, ei, d) for f in feats]
    ref = refcpu.meta_step({k: PT[k] for k in names}, Pg, tasks, list(ml.default_windows()[-1, 0]),
                           cfg.inner_steps, cfg.batch, S, cfg.inner_lr, cfg.max_norm, 1)
    losses = res.losses.cpu().numpy()
    for j in range(2):
        assert rel(losses[:cfg.inner_steps, j], [r[0] for r in ref["step_records"][j]]) < 1e-5
        assert abs(losses[-1, j] - ref["query_losses"][j]) < 1e-4 * ref["query_losses"][j]
        ad = params.unpack(fast[j], d, 0)
        for k in names:
            assert rel(ad[k].cpu().numpy(), ref["adapted"][j][k].numpy()) < 1e-5, k
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), ref["meta_grad"][k].numpy()) < 1e-4, k


# ----------------------------------------------------------------------------- outer AdamW
def test_adamw_matches_torch():
    torch.manual_seed(1)
    d = CONFIG1
    ctx = _capi.Context(d, 0)
    n = 70000
    p0 = torch.randn(n)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-4)
    p = p0.to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for step in range(1, 4):
        g = torch.randn(n) * (3.0 if step == 2 else 0.001)
        ref.grad = g.clone()
        torch.nn.utils.clip_grad_norm_([ref], 1.0)
        opt.step()
        ctx.adamw_step(_capi.stream_ptr(torch), p, g.to(DEV), m, v, step, 1e-3, (0.9, 0.999), 1e-8, 1e-4, 1.0)
    assert rel(p.cpu().numpy(), ref.detach().numpy()) < 1e-6


# ----------------------------------------------------------------------------- properties
def test_determinism_and_task_independence():
    """Bitwise: two identical meta-steps agree; a task's result does not depend on which
    other tasks share its launches (per-task fast weights, fixed-order reductions)."""
    d = ModelDims(num_nodes=49, hidden_channels=64, lstm_hidden_size=64, lstm_num_layers=2)
    cfg = MamlConfig(inner_steps=2, batch=3, order=1)
    P = synth.init_params(9, d, gcn_bias_scale=0.1)
    theta, gcn, _ = split(P)
    ei = grid_edges(d)
    T = stream_len_for(cfg, d)
    feats = [synth.make_features(1000 + j, d.num_nodes, T) for j in range(3)]

    def run(fs, z_pick):
        ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
        ml.set_tasks(fs)
        fast = torch.zeros(len(fs), ml.theta.numel(), device=DEV)
        res = ml.meta_step(fast_out=fast)
        return res.losses[:, z_pick].cpu(), fast[z_pick].cpu()

    l1, f1 = run(feats, 1)
    l2, f2 = run(feats, 1)
    assert torch.equal(l1, l2) and torch.equal(f1, f2)
    l3, f3 = run([feats[1]], 0)
    assert torch.equal(l1, l3) and torch.equal(f1, f3)


def test_full_size_meta_step_properties():
    """BASELINE config 2 shapes (15 tasks x B=32 x T=24 x N=441, K=5): finite losses,
    support losses decrease on average, query MSE close to the target variance at init,
    theta moves, meta-grad finite."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=5, batch=32, order=1)
    P = synth.init_params(42, d)
    theta, gcn, _ = split(P)
    ei = grid_edges(d)
    T = stream_len_for(cfg, d)
    feats = [synth.make_features(synth.task_seed(j), d.num_nodes, T) for j in range(15)]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml.set_tasks(feats)
    theta0 = ml.theta.clone()
    res = ml.meta_step()
    L = res.losses.cpu().numpy()
    assert np.isfinite(L).all()
    assert np.isfinite(ml.meta_grad.cpu().numpy()).all()
    assert 0.5 < L[-1].mean() < 2.0
    assert not torch.equal(theta0, ml.theta)
    assert np.isfinite(res.meta_loss)


# ----------------------------------------------------------------------------- second order
# SMAML_KEEP caps how many inner steps keep their primal activations for the second-order
# sweep (tangent-only dual kernels there); unset = as many as fit (all of them at these sizes).
KEEP_MODES = [None, "0", "1"]


def set_keep(monkeypatch, keep):
    if keep is None:
        monkeypatch.delenv("SMAML_KEEP", raising=False)
    else:
        monkeypatch.setenv("SMAML_KEEP", keep)


@pytest.mark.parametrize("keep", KEEP_MODES)
@pytest.mark.parametrize("clip", [0, 1])
def test_second_order_meta_grad_cfg1(golden_dir, clip, keep, monkeypatch):
    """Second-order meta-gradient (through both inner SGD steps, the Hessian of each support
    loss and the clip_grad_norm_ coefficient) vs torch.func through the reference module."""
    set_keep(monkeypatch, keep)
    d = CONFIG1
    z = load(golden_dir, "cfg1_maml.npz")
    steps, batch, support, qb = (int(z[k]) for k in ("steps", "batch", "support", "qbatch"))
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    cfg = MamlConfig(inner_steps=steps, batch=batch, order=2, support_samples=support,
                     max_norm=float(z["max_norms"][clip]))
    ml = MetaLearner(d, cfg, gcn, theta, z["edge_index"], device=DEV)
    feats = [synth.make_features(int(s), d.num_nodes, synth.t_total_for(support + qb)) for s in z["feat_seeds"]]
    ml.set_tasks(feats)
    res = ml.meta_step()
    losses = res.losses.cpu().numpy()
    total = {k: 0.0 for k in names}
    for j in range(len(feats)):
        tag = f"t{j}_c{clip}_o2"
        assert rel(losses[:steps, j], z[tag + "_losses"]) < 1e-5
        assert abs(losses[steps, j] - float(z[tag + "_query"])) < 1e-5 * float(z[tag + "_query"])
        for k in names:
            total[k] = total[k] + z[f"{tag}_metagrad/{k}"]
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), total[k]) < 1e-4, k


@pytest.mark.parametrize("keep", KEEP_MODES)
@pytest.mark.parametrize("max_norm", [1.0, 0.02])
def test_second_order_matches_oracle_cfg2(max_norm, keep, monkeypatch):
    """Config-2 shapes (N=441, Hc=256, LSTM 4x128), K=2 inner steps, B=1, 2 tasks; the sweep
    recomputes every step's primal (keep 0), keeps the last step's (keep 1) or keeps all."""
    set_keep(monkeypatch, keep)
    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=1, order=2, max_norm=max_norm)
    P = synth.init_params(8, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    T = stream_len_for(cfg, d)
    feats = [synth.make_features(1200 + j, d.num_nodes, T) for j in range(2)]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml.set_tasks(feats)
    res = ml.meta_step()
    PT = refcpu.to_torch(P)
    Pg = {k: v for k, v in PT.items() if k not in names}
    S = cfg.inner_steps * cfg.batch
    tasks = [refcpu.TaskData(f, ei, d) for f in feats]
    ref = refcpu.meta_step({k: PT[k] for k in names}, Pg, tasks, list(ml.default_windows()[-1, 0]),
                           cfg.inner_steps, cfg.batch, S, cfg.inner_lr, cfg.max_norm, 2)
    losses = res.losses.cpu().numpy()
    for j in range(2):
        assert abs(losses[-1, j] - ref["query_losses"][j]) < 1e-4 * ref["query_losses"][j]
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), ref["meta_grad"][k].numpy()) < 1e-4, k


# ----------------------------------------------------------------------------- config 5 shapes
def test_second_order_matches_oracle_cfg5():
    """BASELINE config-5 shapes (N=1024 32x32 grid, Hc=512, LSTM 4x128), K=2, B=1, 1 task:
    second-order meta-gradient and query MSE against the oracle."""
    d = CONFIG5
    cfg = MamlConfig(inner_steps=2, batch=1, order=2)
    P = synth.init_params(9, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1300, d.num_nodes, stream_len_for(cfg, d))]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml.set_tasks(feats)
    res = ml.meta_step()
    PT = refcpu.to_torch(P)
    S = cfg.inner_steps * cfg.batch
    ref = refcpu.meta_step({k: PT[k] for k in names}, {k: v for k, v in PT.items() if k not in names},
                           [refcpu.TaskData(feats[0], ei, d)], list(ml.default_windows()[-1, 0]),
                           cfg.inner_steps, cfg.batch, S, cfg.inner_lr, cfg.max_norm, 2)
    q = float(res.losses[-1, 0].item())
    assert abs(q - ref["query_losses"][0]) < 1e-4 * ref["query_losses"][0]
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), ref["meta_grad"][k].numpy()) < 1e-4, k


@pytest.mark.parametrize("order", [1, 2])
def test_task_groups_match_one_pass(order):
    """A rank running its tasks in groups (task_group) gives the one-pass losses and the same
    meta-gradient (summed over groups before the outer step; rounding-level difference)."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=2, order=order)
    P = synth.init_params(10, d)
    theta, gcn, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1400 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(3)]
    out = []
    for g in (None, 2):
        ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, task_group=g)
        ml.set_tasks(feats)
        res = ml.meta_step()
        out.append((res.losses.cpu().numpy(), ml.meta_grad.cpu().numpy(), ml.theta.cpu().numpy()))
    assert rel(out[1][0], out[0][0]) < 1e-6
    assert rel(out[1][1], out[0][1]) < 1e-6
    assert rel(out[1][2], out[0][2]) < 1e-6


# ----------------------------------------------------------------------------- dropout
@pytest.mark.parametrize("order", [1, 2])
def test_dropout_matches_oracle(order):
    """Train-mode dropout at the reference's training rates (STGCN dropout_rate 0.2 after
    conv1-3, lstm_dropout 0.2 between LSTM layers and on the head input), with the HIP path's
    counter-based masks restated in the oracle: per-step losses, query MSE, meta-gradient
    (first and second order: the sweep must reuse each step's masks)."""
    d = CONFIG1
    cfg = MamlConfig(inner_steps=2, batch=2, order=order)
    P = synth.init_params(11, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1500 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(2)]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, dropout=(0.2, 0.2), dropout_seed=5)
    ml.set_tasks(feats, task_ids=[3, 7])
    res = ml.meta_step()
    seed = (5 * 1000003 + 1) & 0xFFFFFFFF  # MetaLearner's seed of its first meta-step
    PT = refcpu.to_torch(P)
    S = cfg.inner_steps * cfg.batch
    ref = refcpu.meta_step({k: PT[k] for k in names}, {k: v for k, v in PT.items() if k not in names},
                           [refcpu.TaskData(f, ei, d) for f in feats], list(ml.default_windows()[-1, 0]),
                           cfg.inner_steps, cfg.batch, S, cfg.inner_lr, cfg.max_norm, order,
                           dropout=(seed, 0.2, 0.2), task_ids=[3, 7])
    losses = res.losses.cpu().numpy()
    for j in range(2):
        steps = [r[0] for r in ref["step_records"][j]]
        assert rel(losses[:cfg.inner_steps, j], steps) < 1e-5
        assert abs(losses[-1, j] - ref["query_losses"][j]) < 1e-5 * ref["query_losses"][j]
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), ref["meta_grad"][k].numpy()) < 1e-4, k
    # the masks matter: without dropout the meta-gradient is a different one
    ml0 = MetaLearner(d, cfg, gcn, theta, ei, device=DEV)
    ml0.set_tasks(feats)
    ml0.meta_step()
    assert rel(ml.meta_grad.cpu().numpy(), ml0.meta_grad.cpu().numpy()) > 0.05


def test_dropout_masks_follow_task_ids_not_groups():
    """A task's masks are keyed by its global id: running the tasks in groups of one gives the
    one-pass losses under dropout."""
    d = CONFIG1
    cfg = MamlConfig(inner_steps=2, batch=2, order=2)
    P = synth.init_params(12, d)
    theta, gcn, _ = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1600 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(3)]
    out = []
    for g in (None, 1):
        ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, task_group=g, dropout=(0.3, 0.2), dropout_seed=9)
        ml.set_tasks(feats, task_ids=[10, 11, 12])
        out.append((ml.meta_step().losses.cpu().numpy(), ml.meta_grad.cpu().numpy()))
    assert rel(out[1][0], out[0][0]) < 1e-6
    assert rel(out[1][1], out[0][1]) < 1e-5


# ----------------------------------------------------------------------------- bench tile configs
# The config-2 bench runs the 128x128-tile k_lstm_bwd_step / k_lstm_bwd_dual; launches under
# `bwd_big_min` (768) 64-row tile units take the 64x64 or split-K variants instead. These tests run every variant against the oracle and
# assert through the library's launch counters (smaml_variant_counts) which ones ran.
_ORACLE = {}


def _oracle_meta_step(key, d, P, names, feats, ei, cfg, qidx):
    if key not in _ORACLE:
        PT = refcpu.to_torch(P)
        S = cfg.inner_steps * cfg.batch
        _ORACLE[key] = refcpu.meta_step({k: PT[k] for k in names}, {k: v for k, v in PT.items() if k not in names},
                                        [refcpu.TaskData(f, ei, d) for f in feats], qidx, cfg.inner_steps,
                                        cfg.batch, S, cfg.inner_lr, cfg.max_norm, cfg.order)
    return _ORACLE[key]


def _check_meta_step(res, ml, ref, d, names, n_tasks, K):
    losses = res.losses.cpu().numpy()
    for j in range(n_tasks):
        assert rel(losses[:K, j], [r[0] for r in ref["step_records"][j]]) < 1e-5
        assert abs(losses[-1, j] - ref["query_losses"][j]) < 1e-4 * ref["query_losses"][j]
    mg = params.unpack(ml.meta_grad, d, 0)
    for k in names:
        assert rel(mg[k].cpu().numpy(), ref["meta_grad"][k].numpy()) < 1e-4, k


@pytest.mark.parametrize("streams", [1, 2])
@pytest.mark.parametrize("keep", [-1, 0, 1])
def test_second_order_bench_tiles_b32(keep, streams):
    """1 task x B=32 x K=2 at config-2 shapes (M = 14,112 sequences): a diagonal with all 4
    layers holds 4 x 111 x 2 = 888 >= 768 64-row tile units, so the bench's 128x128
    k_lstm_bwd_step and k_lstm_bwd_dual run (kept-primal and recomputed-primal forms by `keep`).
    streams 1: the short corner diagonals run the 64x64 tiles; streams 2 (the default bptt_streams):
    every diagonal in two row chunks on side streams, all on the 128x128 tiles. Per-step losses,
    query MSE and the second-order meta-gradient against the oracle (train_hybrid_maml_v5.py:110-184
    + torch autograd)."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=32, order=2)
    P = synth.init_params(13, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1700, d.num_nodes, stream_len_for(cfg, d))]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, task_group=None)
    ml.set_tasks(feats)
    ml.ctx.set_option("keep", keep)
    ml.ctx.set_option("bptt_streams", streams)
    ml.ctx.variant_counts(reset=True)
    res = ml.meta_step()
    vc = ml.ctx.variant_counts()
    assert vc["bwd_big"] > 0 and (vc["bwd_small"] > 0) == (streams == 1), vc
    if keep == 0:
        assert vc["bwd_dual_big"] > 0 and vc["bwd_dual_big_kept"] == 0, vc
    elif keep == 1:
        assert vc["bwd_dual_big"] > 0 and vc["bwd_dual_big_kept"] > 0, vc
    else:
        assert ml.ctx.so_kept_steps() == 2
        assert vc["bwd_dual_big"] == 0 and vc["bwd_dual_big_kept"] > 0, vc
    ref = _oracle_meta_step("b32", d, P, names, feats, ei, cfg, list(ml.default_windows()[-1, 0]))
    _check_meta_step(res, ml, ref, d, names, 1, cfg.inner_steps)


def test_second_order_bench_tiles_b32_dropout():
    """The bench-size tiles with train-mode dropout (0.2 / 0.2: the masked loaders and the
    dropout variants of the 128x128 BPTT and tangent BPTT kernels) against the oracle's restated
    masks: 1 task x B=32 x K=1, second order."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=1, batch=32, order=2)
    P = synth.init_params(15, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1750, d.num_nodes, stream_len_for(cfg, d))]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, task_group=None, dropout=(0.2, 0.2), dropout_seed=9)
    ml.set_tasks(feats, task_ids=[4])
    ml.ctx.variant_counts(reset=True)
    res = ml.meta_step()
    vc = ml.ctx.variant_counts()
    assert vc["fwd_drop"] > 0 and vc["bwd_big"] > 0 and vc["bwd_dual_big"] + vc["bwd_dual_big_kept"] > 0, vc
    seed = (9 * 1000003 + 1) & 0xFFFFFFFF  # MetaLearner's seed of its first meta-step
    PT = refcpu.to_torch(P)
    ref = refcpu.meta_step({k: PT[k] for k in names}, {k: v for k, v in PT.items() if k not in names},
                           [refcpu.TaskData(f, ei, d) for f in feats], list(ml.default_windows()[-1, 0]),
                           cfg.inner_steps, cfg.batch, cfg.inner_steps * cfg.batch, cfg.inner_lr, cfg.max_norm,
                           cfg.order, dropout=(seed, 0.2, 0.2), task_ids=[4])
    _check_meta_step(res, ml, ref, d, names, 1, cfg.inner_steps)


@pytest.mark.parametrize("tiles", ["big", "small", "split", "kw"])
@pytest.mark.parametrize("keep", [-1, 0])
def test_second_order_tile_variants_task_groups(tiles, keep):
    """Every BPTT tile variant forced at config-2 shapes (B=1, K=2, 3 tasks run in task groups
    of 2): 128x128 tiles (the bench's), 64x64 tiles, and the small-grid steps -- split-K part + cell
    pairs (small_kw 0) or one launch with the K split over waves (kernels_small.hip, small_kw 1)."""
    d = CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=1, order=2)
    P = synth.init_params(14, d, gcn_bias_scale=0.1)
    theta, gcn, names = split(P)
    ei = grid_edges(d)
    feats = [synth.make_features(1800 + j, d.num_nodes, stream_len_for(cfg, d)) for j in range(3)]
    ml = MetaLearner(d, cfg, gcn, theta, ei, device=DEV, task_group=2)
    ml.set_tasks(feats)
    assert len(ml._groups) == 2
    big = 0 if tiles == "big" else 1 << 30
    ml.ctx.set_option("bwd_big_min", big)
    ml.ctx.set_option("bwdd_big_min", big)
    ml.ctx.set_option("split_max", 4 if tiles in ("split", "kw") else 1)
    ml.ctx.set_option("small_kw", 1 if tiles == "kw" else 0)
    ml.ctx.set_option("keep", keep)
    ml.ctx.variant_counts(reset=True)
    res = ml.meta_step()
    vc = ml.ctx.variant_counts()
    dual = ("bwd_dual_big" if tiles == "big" else "bwd_dual_small") + ("_kept" if keep else "")
    assert vc[dual] > 0, vc
    if tiles == "big":
        assert vc["bwd_big"] > 0 and vc["bwd_small"] == vc["bwd_split"] == 0, vc
    elif tiles == "small":
        assert vc["bwd_small"] > 0 and vc["bwd_big"] == vc["bwd_split"] == 0 and vc["fwd_split"] == 0, vc
    elif tiles == "split":
        assert vc["bwd_split"] > 0 and vc["fwd_split"] > 0 and vc["bwd_big"] == 0, vc
    else:
        assert vc["bwd_kw"] > 0 and vc["fwd_kw"] > 0 and vc["bwd_split"] == vc["bwd_big"] == 0, vc
    ref = _oracle_meta_step("groups", d, P, names, feats, ei, cfg, list(ml.default_windows()[-1, 0]))
    _check_meta_step(res, ml, ref, d, names, 3, cfg.inner_steps)
