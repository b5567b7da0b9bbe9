"""Generate golden fixtures by running the REFERENCE modules themselves (this container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_fixtures.py [/root/reference]

The reference (Yalt8826/WeatherForecast_STGCN_MAML) is imported unmodified from its
read-only checkout. Absent third-party packages get offline stubs inserted into
``sys.modules`` first:

* ``torch_geometric.nn.GCNConv`` -- a restatement of PyG 2.x GCNConv (glorot ``lin``
  without bias, zero ``bias``, ``add_remaining_self_loops``, symmetric ``gcn_norm``,
  scatter-add at the target). torch_geometric is not vendored and its version is not
  pinned by the reference (requirements.txt), so parity is UNPINNED at this boundary.
* ``torch_geometric.data.Data`` / ``torch_geometric.loader.DataLoader`` -- containers
  (batch_size 1, identical to PyG collation at batch 1).
* ``xarray`` -- an empty module (only used for annotations on this path).

Inputs (features, weights, graph coordinates) come from ``weatherforecast_stgcn_maml_amd.synth``
(numpy PCG64 seeds), so the GPU box regenerates them bit for bit; only the outputs and
the edge_index are stored. Outputs are data only (no reference source travels).
"""
from __future__ import annotations

import copy
import importlib.machinery
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from weatherforecast_stgcn_maml_amd import synth  # noqa: E402
from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2  # noqa: E402

torch.set_num_threads(os.cpu_count() or 1)


# ----------------------------------------------------------------------------- stubs
def _module(name):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    sys.modules[name] = m
    return m


class _Lin(torch.nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(cout, cin))
        a = (6.0 / (cin + cout)) ** 0.5
        torch.nn.init.uniform_(self.weight, -a, a)

    def forward(self, x):
        return x @ self.weight.t()


class GCNConvStub(torch.nn.Module):
    """PyG 2.x GCNConv semantics (see module docstring)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.lin = _Lin(in_channels, out_channels)
        self.bias = torch.nn.Parameter(torch.zeros(out_channels))

    def forward(self, x, edge_index):
        n = x.shape[0]
        ei = edge_index.long()
        keep = ei[0] != ei[1]
        loop = torch.arange(n)
        row = torch.cat([ei[0][keep], loop])
        col = torch.cat([ei[1][keep], loop])
        w = torch.ones(row.numel(), dtype=x.dtype)
        deg = torch.zeros(n, dtype=x.dtype).scatter_add_(0, col, w)
        dinv = deg.pow(-0.5)
        dinv = dinv.masked_fill(torch.isinf(dinv), 0.0)
        norm = dinv[row] * w * dinv[col]
        h = self.lin(x)
        out = torch.zeros(n, self.out_channels, dtype=x.dtype).index_add_(0, col, h[row] * norm[:, None])
        return out + self.bias


class DataStub:
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    def to(self, device):
        return DataStub(**{k: (v.to(device) if torch.is_tensor(v) else v) for k, v in self.__dict__.items()})


class _Recording(torch.utils.data.Dataset):
    """Delegates to the wrapped dataset and records the indices the loader fetches."""

    def __init__(self, ds, record):
        self.ds, self.record = ds, record

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        self.record.append(int(i))
        return self.ds[i]


class DataLoaderStub(torch.utils.data.DataLoader):
    """PyG ``DataLoader`` at batch_size 1: it IS torch's DataLoader (PyG's subclasses it), so the
    sampler and its draws from the global torch RNG are the real ones; the collate returns the
    single ``Data`` object (PyG's Collater at batch 1 yields the same x, edge_index, y).
    ``record`` holds the dataset indices in the order they were fetched."""

    def __init__(self, dataset, batch_size=1, shuffle=False, **kw):
        assert batch_size == 1
        self.record = []
        super().__init__(_Recording(dataset, self.record), batch_size=1, shuffle=shuffle,
                         collate_fn=lambda b: b[0], **kw)


def install_stubs():
    pyg = _module("torch_geometric")
    pyg_nn = _module("torch_geometric.nn")
    pyg_data = _module("torch_geometric.data")
    pyg_loader = _module("torch_geometric.loader")
    pyg.nn, pyg.data, pyg.loader = pyg_nn, pyg_data, pyg_loader
    pyg_nn.GCNConv = GCNConvStub
    pyg_data.Data = DataStub
    pyg_loader.DataLoader = DataLoaderStub
    xr = _module("xarray")
    xr.Dataset = object
    xr.open_dataset = lambda path, *a, **kw: None   # replaced per fixture (validate)
    xr.merge = lambda dss, *a, **kw: None


def import_reference(ref_dir):
    install_stubs()
    sys.path.insert(0, ref_dir)
    import model as ref_model  # noqa
    import hybrid_model as ref_hybrid  # noqa
    import dataset as ref_dataset  # noqa
    import graphBuilder as ref_graph  # noqa
    import embed_utils as ref_embed  # noqa
    import train_hybrid_maml_v5 as ref_train  # noqa
    import adaptive_scheduler as ref_sched  # noqa
    import adapt_hybrid_v5 as ref_adapt  # noqa
    os.environ.setdefault("MPLBACKEND", "Agg")
    import validate_hybrid_v5 as ref_validate  # noqa
    return types.SimpleNamespace(model=ref_model, hybrid=ref_hybrid, dataset=ref_dataset,
                                 graph=ref_graph, embed=ref_embed, train=ref_train, sched=ref_sched,
                                 adapt=ref_adapt, validate=ref_validate)


# ----------------------------------------------------------------------------- helpers
def build_ref_model(R, d, params):
    base = R.model.STGCN(in_channels=d.input_channels, hidden_channels=d.hidden_channels,
                         out_channels=d.output_channels, window_size=d.window_size,
                         forecast_horizon=d.forecast_horizon, dropout_rate=0.0)
    hyb = R.hybrid.HybridSTGCN_LSTM(base_stgcn=base, lstm_hidden_size=d.lstm_hidden_size,
                                    lstm_num_layers=d.lstm_num_layers, lstm_dropout=0.0,
                                    out_channels=d.output_channels,
                                    forecast_horizon=d.forecast_horizon, freeze_base=False)
    sd = hyb.state_dict()
    assert list(sd.keys()) == list(params.keys()), (list(sd.keys()), list(params.keys()))
    hyb.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    return hyb


def grid_ds(d):
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    return types.SimpleNamespace(latitude=types.SimpleNamespace(values=lats),
                                 longitude=types.SimpleNamespace(values=lons))


def trainable_state(model):
    return {k: v.detach().numpy().copy() for k, v in model.state_dict().items()
            if k.startswith(("lstm.", "output_layer."))}


class Recorder:
    def __init__(self):
        self.losses, self.norms = [], []


def patched_inner(R, rec):
    """Record per-step loss and clip total-norm without changing the computation."""
    orig_clip = torch.nn.utils.clip_grad_norm_
    orig_mse = R.train.nn.MSELoss

    class RecMSE(orig_mse):
        def forward(self, a, b):
            out = super().forward(a, b)
            rec.losses.append(float(out))
            return out

    def rec_clip(params, max_norm, *a, **kw):
        tot = orig_clip(params, max_norm, *a, **kw)
        rec.norms.append(float(tot))
        return tot

    return orig_clip, orig_mse, RecMSE, rec_clip


def run_ref_inner(R, model, koppen, support, inner_epochs):
    rec = Recorder()
    orig_clip, orig_mse, RecMSE, rec_clip = patched_inner(R, rec)
    R.train.INNER_EPOCHS_PER_TASK = inner_epochs
    torch.nn.utils.clip_grad_norm_ = rec_clip
    R.train.nn.MSELoss = RecMSE
    try:
        adapted, _ = R.train.inner_loop_v4(model, koppen, support, "cpu")
    finally:
        torch.nn.utils.clip_grad_norm_ = orig_clip
        R.train.nn.MSELoss = orig_mse
    return adapted, rec


# ----------------------------------------------------------------------------- fixtures
def fixture_forward_and_inner(R, d, name, feat_seed, param_seed, n_samples, inner_epochs,
                              n_support, tasks=2, full=True):
    from torch.utils.data import Subset

    params = synth.init_params(param_seed, d, gcn_bias_scale=0.1)
    ds = grid_ds(d)
    ei, n, _ = R.graph.build_spatial_graph(ds, k_neighbors=4)
    assert n == d.num_nodes
    out = {"edge_index": ei.numpy().astype(np.int64),
           "feat_seeds": np.array([feat_seed + j for j in range(tasks)]),
           "param_seed": np.array(param_seed), "n_samples": np.array(n_samples),
           "inner_epochs": np.array(inner_epochs), "n_support": np.array(n_support)}
    model = build_ref_model(R, d, params)
    koppen = R.embed.KoppenEmbedding(embedding_dim=8)
    t_total = synth.t_total_for(n_samples)
    meta_tasks = []
    for j in range(tasks):
        feats = torch.from_numpy(synth.make_features(feat_seed + j, d.num_nodes, t_total))
        dataset = R.dataset.WeatherGraphDataset(feats, ei, window_size=d.window_size,
                                                forecast_horizon=d.forecast_horizon)
        assert len(dataset) == n_samples
        support = Subset(dataset, list(range(0, n_support)))
        query = Subset(dataset, list(range(n_support, n_samples)))
        meta_tasks.append((support, query, None))
        if j == 0:
            s0 = dataset[0]
            model.eval()
            with torch.no_grad():
                feats0 = model.extract_base_features(s0.x, s0.edge_index)
                pred0 = model(s0.x, s0.edge_index)
            out["pred0"] = pred0.numpy()
            out["loss0"] = np.array(float(torch.nn.MSELoss()(pred0, s0.y)))
            if full:
                out["feats0"] = feats0.numpy()
            else:
                out["feats0_rows"] = feats0[:: max(1, feats0.shape[0] // 64)].numpy()
                out["feats0_sum"] = np.array(float(feats0.double().sum()))
                out["feats0_sqsum"] = np.array(float((feats0.double() ** 2).sum()))
        adapted, rec = run_ref_inner(R, model, koppen, support, inner_epochs)
        out[f"t{j}_losses"] = np.array(rec.losses)
        out[f"t{j}_norms"] = np.array(rec.norms)
        ast = trainable_state(adapted)
        if full:
            for k, v in ast.items():
                out[f"t{j}_adapted/{k}"] = v
        else:
            for k, v in ast.items():
                out[f"t{j}_adapted_norm/{k}"] = np.array(float(np.linalg.norm(v.astype(np.float64))))
                out[f"t{j}_adapted_slice/{k}"] = v.reshape(-1)[:64].copy()
        q = query[0]
        adapted.train()
        with torch.no_grad():
            out[f"t{j}_query_mse"] = np.array(float(torch.nn.MSELoss()(adapted(q.x, q.edge_index), q.y)))
    # the reference's own meta_update_v4 (outer update is a no-op, F1)
    opt = torch.optim.AdamW(list(model.parameters()) + list(koppen.parameters()), lr=1e-3,
                            weight_decay=1e-4)
    before = {k: v.clone() for k, v in model.state_dict().items()}
    R.train.INNER_EPOCHS_PER_TASK = inner_epochs
    out["meta_loss"] = np.array(R.train.meta_update_v4(model, koppen, meta_tasks, "cpu", opt))
    out["meta_noop"] = np.array(all(torch.equal(before[k], v) for k, v in model.state_dict().items()))
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **out)
    print("wrote", path, "meta_loss", float(out["meta_loss"]), "noop", bool(out["meta_noop"]))


def fixture_maml(R, d, name, feat_seed, param_seed, steps, batch, support, qbatch,
                 max_norms=(1.0, 0.05), tasks=2):
    """FO and second-order meta-gradients through the reference module via torch.func."""
    from torch.func import functional_call

    params = synth.init_params(param_seed, d, gcn_bias_scale=0.1)
    model = build_ref_model(R, d, params)
    model.train()
    ds = grid_ds(d)
    ei, _, _ = R.graph.build_spatial_graph(ds, k_neighbors=4)
    n_samples = support + qbatch
    t_total = synth.t_total_for(n_samples)
    crit = torch.nn.MSELoss()
    names = [k for k in params if k.startswith(("lstm.", "output_layer."))]
    frozen = {k: torch.from_numpy(v) for k, v in params.items() if k not in names}
    out = {"edge_index": ei.numpy().astype(np.int64), "param_seed": np.array(param_seed),
           "feat_seeds": np.array([feat_seed + j for j in range(tasks)]),
           "steps": np.array(steps), "batch": np.array(batch), "support": np.array(support),
           "qbatch": np.array(qbatch), "max_norms": np.array(max_norms)}
    for j in range(tasks):
        feats = torch.from_numpy(synth.make_features(feat_seed + j, d.num_nodes, t_total))
        dataset = R.dataset.WeatherGraphDataset(feats, ei, window_size=d.window_size,
                                                forecast_horizon=d.forecast_horizon)
        samples = [dataset[i] for i in range(n_samples)]

        def loss_fn(theta, idx):
            full = dict(frozen)
            full.update(theta)
            ls = [crit(functional_call(model, full, (samples[i].x, samples[i].edge_index)),
                       samples[i].y) for i in idx]
            return torch.stack(ls).mean()

        for mi, mx in enumerate(max_norms):
            for order in (1, 2):
                theta0 = {k: torch.from_numpy(params[k]).clone().requires_grad_(True) for k in names}
                theta = dict(theta0)
                losses, norms = [], []
                for k in range(steps):
                    idx = [(k * batch + b) % support for b in range(batch)]
                    L = loss_fn(theta, idx)
                    g = torch.autograd.grad(L, list(theta.values()), create_graph=(order == 2))
                    tot = torch.stack([gi.norm(2) for gi in g]).norm(2)
                    coef = torch.clamp(mx / (tot + 1e-6), max=1.0)
                    theta = {kk: v - 0.01 * coef * gi for (kk, v), gi in zip(theta.items(), g)}
                    if order == 1:
                        theta = {kk: v.detach().requires_grad_(True) for kk, v in theta.items()}
                    losses.append(float(L))
                    norms.append(float(tot))
                qidx = list(range(support, support + qbatch))
                Lq = loss_fn(theta, qidx) * 0.5
                wrt = list(theta0.values()) if order == 2 else list(theta.values())
                mg = torch.autograd.grad(Lq, wrt)
                tag = f"t{j}_c{mi}_o{order}"
                out[tag + "_losses"] = np.array(losses)
                out[tag + "_norms"] = np.array(norms)
                out[tag + "_query"] = np.array(float(Lq) / 0.5)
                for kk, gi in zip(names, mg):
                    out[f"{tag}_metagrad/{kk}"] = gi.detach().numpy().copy()
                if order == 1:
                    for kk, v in theta.items():
                        out[f"{tag}_adapted/{kk}"] = v.detach().numpy().copy()
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **out)
    print("wrote", path)


class _GridDS:
    """The xarray Dataset surface adaptModel touches: coordinates for build_spatial_graph,
    ``sizes`` for a print, and ``"day_of_year_sin" in ds`` (time features already present)."""

    def __init__(self, d):
        g = grid_ds(d)
        self.latitude, self.longitude, self.sizes = g.latitude, g.longitude, {}

    def __contains__(self, key):
        return True


def fixture_adapt(R, d, name, feat_seed, param_seed, n_samples, regions, sched_losses):
    """adapt_hybrid_v5.adaptModel run UNMODIFIED on synthetic data (adapt_hybrid_v5.py:65-271):
    the ERA5 loader / preprocessing are replaced by a synthetic feature stream, the checkpoint
    load by an in-memory dict, torch.save by a capture; dropout is set to 0 (the parity setting:
    STGCN dropout_rate, hard-coded 0.2 at :106, is overridden, lstm_dropout comes from the
    checkpoint's hybrid_config). Records the per-epoch shuffle orders, per-step train losses,
    the scheduler's learning rates, the validation MSE and the adapted parameters. Also pins
    ClimateAwareLRScheduler / create_climate_optimizer (adaptive_scheduler.py:7-94) directly."""
    import tempfile

    params = synth.init_params(param_seed, d, gcn_bias_scale=0.1)
    feats = torch.from_numpy(synth.make_features(feat_seed, d.num_nodes, synth.t_total_for(n_samples)))
    out = {"param_seed": np.array(param_seed), "feat_seed": np.array(feat_seed), "n_samples": np.array(n_samples),
           "regions": np.array(regions), "sched_losses": np.array(sched_losses)}
    # -- the scheduler and optimizer factory on their own
    for region in regions:
        opt, lr0 = R.sched.create_climate_optimizer([torch.nn.Parameter(torch.zeros(1))], region)
        sch = R.sched.ClimateAwareLRScheduler(opt, region, lr0)
        out[f"sched/{region}/lr0"] = np.array(lr0)
        out[f"sched/{region}/wd"] = np.array(opt.param_groups[0]["weight_decay"])
        out[f"sched/{region}/lrs"] = np.array([sch.step(x) for x in sched_losses])
    # -- the full adaptation loop
    ckpt = {"config": {"input_channels": d.input_channels, "hidden_channels": d.hidden_channels,
                       "output_channels": d.output_channels, "window_size": d.window_size,
                       "forecast_horizon": d.forecast_horizon},
            "hybrid_config": {"lstm_hidden_size": d.lstm_hidden_size, "lstm_num_layers": d.lstm_num_layers,
                              "lstm_dropout": 0.0},
            "hybrid_model_state_dict": {k: torch.from_numpy(v) for k, v in params.items()},
            "koppen_embed_state_dict": {"embedding.weight": torch.zeros(31, 8)},
            "model_version": "5.0", "total_params": int(sum(v.size for v in params.values()))}
    stats = {"mean": np.zeros(12), "std": np.ones(12)}
    saved, losses, loaders = {}, [], []
    orig = dict(load=torch.load, save=torch.save, mse=torch.nn.MSELoss, stgcn=R.adapt.STGCN,
                lda=R.adapt.load_adaptation_data, pmi=R.adapt.prepare_model_input,
                sched=R.adapt.ClimateAwareLRScheduler, dl=R.adapt.DataLoader)

    class RecMSE(orig["mse"]):
        def forward(self, a, b):
            out_ = super().forward(a, b)
            losses.append(float(out_))
            return out_

    class RecSched(orig["sched"]):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            self.calls = []
            saved["sched"] = self

        def step(self, epoch_loss=None):
            lr = super().step(epoch_loss)
            self.calls.append((epoch_loss, lr))
            return lr

    class RecLoader(orig["dl"]):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            loaders.append(self)

    for region in regions:
        saved.clear()
        losses.clear()
        loaders.clear()
        torch.load = lambda *a, **kw: ckpt
        torch.save = lambda obj, path: saved.__setitem__("ckpt", obj)
        torch.nn.MSELoss = RecMSE
        R.adapt.STGCN = lambda **kw: orig["stgcn"](**dict(kw, dropout_rate=0.0))
        R.adapt.load_adaptation_data = lambda coords: _GridDS(d)
        R.adapt.prepare_model_input = lambda ds, code, emb, normalize=True, stats=None: (feats, stats_)
        R.adapt.ClimateAwareLRScheduler = RecSched
        R.adapt.DataLoader = RecLoader
        stats_ = stats
        cwd = os.getcwd()
        try:
            with tempfile.TemporaryDirectory() as tmp:
                os.chdir(tmp)
                torch.manual_seed(0)
                R.adapt.adaptModel((18, 23, 75, 80), region)
        finally:
            os.chdir(cwd)
            torch.load, torch.save, torch.nn.MSELoss = orig["load"], orig["save"], orig["mse"]
            R.adapt.STGCN, R.adapt.load_adaptation_data = orig["stgcn"], orig["lda"]
            R.adapt.prepare_model_input, R.adapt.ClimateAwareLRScheduler = orig["pmi"], orig["sched"]
            R.adapt.DataLoader = orig["dl"]
        train, val = loaders[0], loaders[1]
        n_train, epochs = len(train.dataset), len(saved["sched"].calls)
        order = np.array(train.record).reshape(epochs, n_train)
        tag = f"adapt/{region}"
        out[tag + "/orders"] = order
        out[tag + "/train_losses"] = np.array(losses[:epochs * n_train]).reshape(epochs, n_train)
        out[tag + "/val_losses"] = np.array(losses[epochs * n_train:])
        out[tag + "/sched_calls"] = np.array(saved["sched"].calls)
        out[tag + "/val_loss"] = np.array(saved["ckpt"]["val_loss"])
        assert np.array(val.record).tolist() == list(range(len(val.dataset)))
        for k, v in saved["ckpt"]["hybrid_model_state_dict"].items():
            if k.startswith(("lstm.", "output_layer.")):
                out[f"{tag}/adapted/{k}"] = v.numpy().copy()
            else:  # the frozen GCN stack (no grads, F2) must come back unchanged
                assert torch.equal(v, torch.from_numpy(params[k])), k
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **out)
    print("wrote", path)


class _Times:
    def __init__(self, values):
        self.values = values

    def __len__(self):
        return len(self.values)


class _ValDS(_GridDS):
    """The xarray surface validateAdapted touches (validate_hybrid_v5.py:137-170): region and
    time selection, ``valid_time`` timestamps, ``"day_of_year_sin" in ds``."""

    def __init__(self, d, n_times):
        super().__init__(d)
        self.valid_time = _Times(np.datetime64("2025-01-01T00") + np.arange(n_times).astype("timedelta64[h]"))

    def sel(self, **kw):
        return self

    def isel(self, valid_time):
        out = _ValDS.__new__(_ValDS)
        out.__dict__.update(self.__dict__)
        out.valid_time = _Times(self.valid_time.values[valid_time])
        return out

    def __getitem__(self, key):
        return self.valid_time


def fixture_validate(R, d, name, feat_seed, param_seed, n_times):
    """validate_hybrid_v5.validateAdapted run UNMODIFIED on synthetic data (:113-371): the 2025
    NetCDF reads are replaced by a coordinate/time surface, the checkpoint load by an in-memory
    adapted checkpoint (with normalisation stats), prepare_model_input by the synthetic feature
    stream of the selected time slice; plots go to a temporary directory. Records the returned
    denormalised per-variable MSE / MAE and the average (sp excluded)."""
    import tempfile

    params = synth.init_params(param_seed, d, gcn_bias_scale=0.1)
    T0 = max(0, n_times // 4)
    T_sub = min(n_times, T0 + 50) - T0
    feats = torch.from_numpy(synth.make_features(feat_seed, d.num_nodes, T_sub))
    rng = np.random.default_rng(param_seed + 1)
    stats = {"mean": np.array([1.5, -0.8, 285.0, 278.0, 101300.0, 0.0004, 2.1, -1.1, 3.0e5, 0.4, 0.5, -1e-5]),
             "std": np.abs(rng.normal(size=12)) * np.array([3, 3, 8, 7, 900, 1e-3, 4, 4, 1e5, 0.3, 0.3, 1e-4]) + 1e-3}
    ckpt = {"config": {"input_channels": d.input_channels, "hidden_channels": d.hidden_channels,
                       "output_channels": d.output_channels, "window_size": d.window_size,
                       "forecast_horizon": d.forecast_horizon},
            "hybrid_config": {"lstm_hidden_size": d.lstm_hidden_size, "lstm_num_layers": d.lstm_num_layers,
                              "lstm_dropout": 0.2},
            "hybrid_model_state_dict": {k: torch.from_numpy(v) for k, v in params.items()},
            "koppen_embed_state_dict": {"embedding.weight": torch.zeros(31, 8)}, "stats": stats}
    V = R.validate
    orig = dict(load=torch.load, open=V.xr.open_dataset, merge=V.xr.merge, pmi=V.prepare_model_input)
    region, coords = "NewYork2025", (40, 45, 285, 290)
    cwd = os.getcwd()
    try:
        with tempfile.TemporaryDirectory() as tmp:
            os.chdir(tmp)
            os.makedirs("Out_Data/AdaptedModels")
            open(f"Out_Data/AdaptedModels/hybrid_v5_adapted_{region}_{coords}.pt", "wb").close()
            torch.load = lambda *a, **kw: ckpt
            V.xr.open_dataset = lambda path, *a, **kw: _ValDS(d, n_times)
            V.xr.merge = lambda dss, *a, **kw: dss[0]
            V.prepare_model_input = lambda ds, code, emb, normalize=True, stats=None: (feats, stats)
            res = V.validateAdapted(coords, region)
    finally:
        os.chdir(cwd)
        torch.load, V.xr.open_dataset, V.xr.merge = orig["load"], orig["open"], orig["merge"]
        V.prepare_model_input = orig["pmi"]
    out = {"param_seed": np.array(param_seed), "feat_seed": np.array(feat_seed), "n_times": np.array(n_times),
           "t_sub": np.array(T_sub), "stats_mean": stats["mean"], "stats_std": stats["std"],
           "average_mse": np.array(res["average_mse"]), "var_names": np.array(list(V.VAR_NAMES[:6]))}
    for v in V.VAR_NAMES[:6]:
        out[f"{v}/mse"] = np.array(res[v]["mse"])
        out[f"{v}/mae"] = np.array(res[v]["mae"])
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **out)
    print("wrote", path, "average_mse", float(res["average_mse"]))


def fixture_stgcn_forward(R, name, dims_list, param_seed, feat_seed):
    """model.STGCN.forward (model.py:30-52) in eval mode: conv1..4 + ReLU (+ dropout, off in
    eval), last time block, output_layer, view(N, Hf, C).reshape(-1, C)."""
    out = {"param_seed": np.array(param_seed), "feat_seed": np.array(feat_seed)}
    for i, d in enumerate(dims_list):
        params = synth.init_params(param_seed, d, gcn_bias_scale=0.1)
        base = R.model.STGCN(in_channels=d.input_channels, hidden_channels=d.hidden_channels,
                             out_channels=d.output_channels, window_size=d.window_size,
                             forecast_horizon=d.forecast_horizon, dropout_rate=0.2)
        base.load_state_dict({k[len("base_stgcn."):]: torch.from_numpy(v) for k, v in params.items()
                              if k.startswith("base_stgcn.")})
        base.eval()
        ei, _, _ = R.graph.build_spatial_graph(grid_ds(d), k_neighbors=4)
        x, _ = synth.sample_xy(synth.make_features(feat_seed, d.num_nodes, synth.t_total_for(1)), 0)
        with torch.no_grad():
            y = base(torch.from_numpy(np.ascontiguousarray(x)), ei)
        out[f"d{i}/num_nodes"] = np.array(d.num_nodes)
        out[f"d{i}/hidden_channels"] = np.array(d.hidden_channels)
        out[f"d{i}/edge_index"] = ei.numpy().astype(np.int64)
        out[f"d{i}/out"] = y.numpy()
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **out)
    print("wrote", path)


def main():
    ref_dir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    which = sys.argv[2:] or ["cfg1", "maml", "cfg2", "adapt", "stgcn", "validate"]
    R = import_reference(ref_dir)
    torch.manual_seed(0)
    if "cfg1" in which:
        fixture_forward_and_inner(R, CONFIG1, "cfg1_ref.npz", feat_seed=1000, param_seed=7,
                                  n_samples=20, inner_epochs=6, n_support=15, tasks=2, full=True)
    if "maml" in which:
        fixture_maml(R, CONFIG1, "cfg1_maml.npz", feat_seed=2000, param_seed=11, steps=2,
                     batch=3, support=6, qbatch=3)
    if "cfg2" in which:
        fixture_forward_and_inner(R, CONFIG2, "cfg2_ref.npz", feat_seed=1000, param_seed=42,
                                  n_samples=4, inner_epochs=1, n_support=3, tasks=1, full=False)
    if "adapt" in which:
        fixture_adapt(R, CONFIG1, "cfg4_adapt.npz", feat_seed=4000, param_seed=17, n_samples=20,
                      regions=["Thailand", "Moscow", "Delhi"],
                      sched_losses=[1.4, 1.2, 0.9, 1.3, 0.15, 0.5, 1.1, 0.1, 0.7, 1.05, 0.19, 0.3, 2.0, 0.9, 0.05])
    if "validate" in which:
        fixture_validate(R, CONFIG1, "cfg1_validate.npz", feat_seed=4200, param_seed=29, n_times=160)
        fixture_validate(R, CONFIG2, "cfg2_validate.npz", feat_seed=4300, param_seed=31, n_times=160)
    if "stgcn" in which:
        fixture_stgcn_forward(R, "stgcn_forward.npz", [CONFIG1, CONFIG2], param_seed=23, feat_seed=4100)


if __name__ == "__main__":
    main()
