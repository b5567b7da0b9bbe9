"""Regional adaptation (adapt_hybrid_v5.adaptModel, BASELINE config 4) on the GPU vs the CPU
oracle's restatement of the same loop (batch-1 shuffled Adam + clip + climate LR schedule)."""
import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import checkpoint, params, synth
from weatherforecast_stgcn_maml_amd.adapt import adapt
from weatherforecast_stgcn_maml_amd.config import CONFIG1
from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("region,drop", [("Thailand", None), ("Delhi", None), ("Delhi", (0.2, 0.2))])
def test_adaptation_matches_oracle(region, drop, tmp_path):
    """drop: train-mode dropout at the reference's rates with the oracle's restated masks."""
    d = CONFIG1
    P = synth.init_params(21, d, gcn_bias_scale=0.1)
    tr = {k: v for k, v in P.items() if k.startswith(("lstm.", "output_layer."))}
    gcn = {k: v for k, v in P.items() if k not in tr}
    lats, lons = synth.region_grid(n_lat=5, n_lon=5)
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(3100, d.num_nodes, synth.t_total_for(20))
    epochs = 5
    torch.manual_seed(123)
    res = adapt(d, feats, ei, {k: v for k, v in gcn.items() if k.startswith("base_stgcn.conv")}, tr, region,
                epochs=epochs, device="cuda:0", dropout=drop or (0.0, 0.0), dropout_seed=77)
    torch.manual_seed(123)
    PT = refcpu.to_torch(P)
    ref_p, ref_losses, ref_lrs, ref_val, _ = refcpu.adapt_reference(
        {k: PT[k] for k in tr}, {k: v for k, v in PT.items() if k not in tr}, refcpu.TaskData(feats, ei, d),
        region, epochs, dropout=(77, drop[0], drop[1]) if drop else None)
    assert res.n_train == 16 and res.n_val == 4
    np.testing.assert_allclose(res.lrs, ref_lrs, rtol=1e-12)
    assert rel(res.epoch_losses, ref_losses) < 1e-5
    got = params.unpack(res.theta, d, 0)
    for k in tr:
        assert rel(got[k].cpu().numpy(), ref_p[k].numpy()) < 1e-5, k
    assert abs(res.val_loss - ref_val) < 1e-5 * ref_val
    ck = checkpoint.adapted_checkpoint(d, gcn, res.theta, {"embedding.weight": torch.zeros(31, 8)},
                                       (18, 23, 75, 80), region, {"mean": np.zeros(12), "std": np.ones(12)},
                                       res.val_loss)
    checkpoint.save(ck, str(tmp_path / "adapted.pt"))
    back = checkpoint.load(str(tmp_path / "adapted.pt"), weights_only=False)  # our own file (numpy stats)
    assert back["adaptation_type"] == "v5_regional_adaptation_adaptive" and back["region_name"] == region


def _split(P):
    tr = {k: v for k, v in P.items() if k.startswith(("lstm.", "output_layer."))}
    return tr, {k: v for k, v in P.items() if k not in tr}


@pytest.mark.parametrize("region", ["Thailand", "Moscow", "Delhi"])
def test_adaptation_matches_reference_adapt_model(golden_dir, region):
    """adapt() on the GPU against adapt_hybrid_v5.adaptModel run unmodified on the same
    synthetic stream (tests/golden/cfg4_adapt.npz; the recorded DataLoader shuffle orders
    replayed): per-step and per-epoch losses, learning rates, validation MSE, adapted params."""
    import os
    z = np.load(os.path.join(golden_dir, "cfg4_adapt.npz"))
    d = CONFIG1
    P = synth.init_params(int(z["param_seed"]), d, gcn_bias_scale=0.1)
    tr, gcn = _split(P)
    lats, lons = synth.region_grid(n_lat=5, n_lon=5)
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(int(z["feat_seed"]), d.num_nodes, synth.t_total_for(int(z["n_samples"])))
    tag = f"adapt/{region}"
    orders = z[tag + "/orders"]
    res = adapt(d, feats, ei, {k: v for k, v in gcn.items() if k.startswith("base_stgcn.conv")}, tr, region,
                epochs=len(orders), device="cuda:0", orders=orders)
    calls = z[tag + "/sched_calls"]
    assert rel(res.epoch_losses, calls[:, 0]) < 1e-5
    np.testing.assert_allclose(res.lrs, [float(z[f"sched/{region}/lr0"])] + list(calls[:-1, 1]), rtol=1e-6)
    assert abs(res.val_loss - float(z[tag + "/val_loss"])) < 1e-5 * float(z[tag + "/val_loss"])
    got = params.unpack(res.theta, d, 0)
    for k in tr:
        assert rel(got[k].cpu().numpy(), z[f"{tag}/adapted/{k}"]) < 1e-5, k


@pytest.mark.parametrize("small_kw", [0, 1, 2], ids=["split-k", "kw", "kw-bwd-img"])
def test_adaptation_n441_matches_oracle(small_kw):
    """BASELINE config 4 shapes (N=441, Hc=256, LSTM 4x128, batch-1 steps): 2 epochs over 16
    shuffled training windows + the 4-window validation, against the oracle. Runs the
    small-grid forward / BPTT steps -- the split-K part + cell launch pairs (small_kw 0) or the
    one-launch K-split-over-waves kernels (kernels_small.hip, small_kw 1; 2 with the BPTT's pre-split
    weight images) -- and the per-window GCN
    feature cache (the second epoch reads every window's features from it)."""
    from weatherforecast_stgcn_maml_amd import _capi
    from weatherforecast_stgcn_maml_amd.config import CONFIG2

    d = CONFIG2
    P = synth.init_params(22, d, gcn_bias_scale=0.1)
    tr, gcn = _split(P)
    lats, lons = synth.region_grid()
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(3200, d.num_nodes, synth.t_total_for(20))
    ctx = _capi.Context(d, 0)
    ctx.set_option("small_kw", small_kw)
    ctx.variant_counts(reset=True)
    torch.manual_seed(5)
    res = adapt(d, feats, ei, {k: v for k, v in gcn.items() if k.startswith("base_stgcn.conv")}, tr, "Moscow",
                epochs=2, device="cuda:0", ctx=ctx)
    vc = ctx.variant_counts()
    if small_kw:
        assert vc["fwd_kw"] > 0 and vc["bwd_kw"] > 0 and vc["fwd_split"] == 0 and vc["bwd_split"] == 0, vc
    else:
        assert vc["fwd_split"] > 0 and vc["bwd_split"] > 0 and vc["fwd_kw"] == 0 and vc["bwd_kw"] == 0, vc
    torch.manual_seed(5)
    PT = refcpu.to_torch(P)
    tr_t, gcn_t = _split(PT)
    ref_p, ref_losses, ref_lrs, ref_val, _ = refcpu.adapt_reference(tr_t, gcn_t, refcpu.TaskData(feats, ei, d),
                                                                    "Moscow", 2)
    assert res.n_train == 16 and res.n_val == 4
    np.testing.assert_allclose(res.lrs, ref_lrs, rtol=1e-12)
    assert rel(res.epoch_losses, ref_losses) < 1e-5
    got = params.unpack(res.theta, d, 0)
    for k in tr:
        assert rel(got[k].cpu().numpy(), ref_p[k].numpy()) < 1e-5, k
    assert abs(res.val_loss - ref_val) < 1e-5 * ref_val



def test_adaptation_cache_fill_batched_bitwise():
    """The adaptation feature cache filled up front in runs of consecutive windows, each run as one
    GCN pass over single-window tasks (api.cpp ad_cache_fill, option adapt_gcn_batch), against the
    per-step fill (adapt_gcn_batch 0): bitwise the same features, so bitwise the same adaptation
    (config-4 shapes, 2 epochs over 16 shuffled windows; runs of 16 and of <= 3 windows)."""
    from weatherforecast_stgcn_maml_amd import _capi
    from weatherforecast_stgcn_maml_amd.config import CONFIG2

    d = CONFIG2
    P = synth.init_params(23, d, gcn_bias_scale=0.1)
    tr, gcn = _split(P)
    lats, lons = synth.region_grid()
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = synth.make_features(3300, d.num_nodes, synth.t_total_for(20))
    out = {}
    for nb in (0, 32, 3):
        ctx = _capi.Context(d, 0)
        ctx.set_option("adapt_gcn_batch", nb)
        torch.manual_seed(9)
        res = adapt(d, feats, ei, {k: v for k, v in gcn.items() if k.startswith("base_stgcn.conv")}, tr, "Moscow",
                    epochs=2, device="cuda:0", ctx=ctx)
        out[nb] = (res.theta.cpu().numpy(), res.epoch_losses, res.val_loss)
        ctx.close()
    for nb in (32, 3):
        assert np.array_equal(out[nb][0], out[0][0]), nb
        assert out[nb][1] == out[0][1] and out[nb][2] == out[0][2], nb


def test_adapt_prepare_phases_and_cache_invalidation():
    """smaml_adapt_prepare allocates the workspace and the per-window feature cache before any epoch
    (adaptModel's set-up, adapt_hybrid_v5.py:163-181), so the epochs allocate nothing; the phase report
    (smaml_adapt_phases) shows the batched cache fill in the first epoch only; a new set of GCN
    parameters invalidates the cached windows without freeing them, and the next epoch refills them:
    bitwise the same losses and parameters as a fresh context."""
    from weatherforecast_stgcn_maml_amd import _capi, adapt as adapt_mod
    from weatherforecast_stgcn_maml_amd.config import CONFIG2

    d = CONFIG2
    P = synth.init_params(25, d, gcn_bias_scale=0.1)
    tr, gcn = _split(P)
    lats, lons = synth.region_grid()
    ei = build_spatial_graph(lats, lons, 4)[0]
    feats = torch.from_numpy(np.ascontiguousarray(synth.make_features(3500, d.num_nodes, synth.t_total_for(24)))).cuda()
    dev = torch.device("cuda:0")
    stream = _capi.stream_ptr(torch)
    order = np.random.default_rng(5).permutation(16).astype(np.int32).reshape(-1, 1)
    lr_dev = torch.full((16,), 1e-3, device=dev)
    gflat = params.pack({k: v for k, v in gcn.items() if k.startswith("base_stgcn.conv")}, d, which=1, device=dev)

    def fresh_ctx():
        ctx = _capi.Context(d, 0)
        ctx.set_graph(ei)
        ctx.set_gcn_params(gflat)
        ctx.set_tasks([feats])
        ctx.set_task_ids([0])
        ctx.set_option("adapt_phase_sync", 1)
        return ctx

    def epoch(ctx, th, m, v, step):
        losses = torch.empty(16, device=dev)
        ctx.adapt_steps(stream, th, m, v, step, order, lr_dev, (0.9, 0.999), 1e-8, 0.0, adapt_mod.MAX_GRAD_NORM,
                        losses)
        torch.cuda.synchronize()
        return losses.cpu().numpy(), ctx.adapt_phases()

    th0 = params.pack(tr, d, which=0, device=dev)
    ctx = fresh_ctx()
    ctx.adapt_prepare(stream, 1)
    prep = ctx.adapt_phases()
    assert prep["cache_alloc_ms"] > 0.0
    ctx.adapt_prepare(stream, 1)  # already prepared: nothing allocated (the phase is the timer's own cost)
    assert ctx.adapt_phases()["cache_alloc_ms"] < 0.5
    th, m, v = th0.clone(), torch.zeros_like(th0), torch.zeros_like(th0)
    l1, ph1 = epoch(ctx, th, m, v, 0)
    l2, ph2 = epoch(ctx, th, m, v, 16)
    for ph in (ph1, ph2):
        assert ph["reserve_ms"] < 0.5 and ph["cache_alloc_ms"] < 0.5 and ph["windows_filled_per_step"] == 0, ph
    assert ph1["cache_fill_ms"] > ph2["cache_fill_ms"], (ph1, ph2)  # epoch 2 reads the cache
    ctx.set_gcn_params(gflat)  # (same values, but the cache must not be trusted: refilled, not reallocated)
    l3, ph3 = epoch(ctx, th, m, v, 32)
    assert ph3["cache_alloc_ms"] < 0.5 and ph3["cache_fill_ms"] > ph2["cache_fill_ms"], (ph2, ph3)
    got = (l1, l2, l3, th.cpu().numpy())
    ctx.close()
    # the same three epochs on a fresh context without adapt_prepare (the first call allocates)
    ctx = fresh_ctx()
    th, m, v = th0.clone(), torch.zeros_like(th0), torch.zeros_like(th0)
    ref = [epoch(ctx, th, m, v, s)[0] for s in (0, 16, 32)] + [th.cpu().numpy()]
    ctx.close()
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
