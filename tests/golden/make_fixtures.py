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


class DataLoaderStub:
    def __init__(self, ds, batch_size=1, shuffle=False, **kw):
        assert batch_size == 1
        self.ds, self.shuffle = ds, shuffle

    def __iter__(self):
        order = torch.randperm(len(self.ds)).tolist() if self.shuffle else range(len(self.ds))
        for i in order:
            yield self.ds[i]

    def __len__(self):
        return len(self.ds)


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


def import_reference(ref_dir):
    install_stubs()
    sys.path.insert(0, ref_dir)
    import model as ref_model  # noqa
    import hybrid_model as ref_hybrid  # noqa
    import dataset as ref_dataset  # noqa
    import graphBuilder as ref_graph  # noqa
    import embed_utils as ref_embed  # noqa
    import train_hybrid_maml_v5 as ref_train  # noqa
    return types.SimpleNamespace(model=ref_model, hybrid=ref_hybrid, dataset=ref_dataset,
                                 graph=ref_graph, embed=ref_embed, train=ref_train)


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


def main():
    ref_dir = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    which = sys.argv[2:] or ["cfg1", "maml", "cfg2"]
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


if __name__ == "__main__":
    main()
