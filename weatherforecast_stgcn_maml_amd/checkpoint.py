"""Checkpoint dicts in the reference's layout.

Meta-training checkpoints follow ``train_hybrid_maml_v5.py:311-335`` (best) and ``:345-370``
(final): ``hybrid_model_state_dict``, ``koppen_embed_state_dict``,
``meta_optimizer_state_dict`` (torch AdamW format over hybrid params + Köppen, in the
reference's parameter order), ``scheduler_state_dict`` (CosineAnnealingWarmRestarts),
``epoch``, ``best_loss`` (+ ``final_loss``), ``model_version``, ``total_params``,
``config`` and ``hybrid_config``. Adapted checkpoints (``adapt_hybrid_v5.py:240-257``) add
``region``, ``region_name``, ``climate_type``, ``stats``, ``adaptation_type``, ``val_loss``,
``base_model_loss``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import params, synth
from .config import ModelDims

MODEL_VERSION = "5.0"


def _t(v):
    return v.detach().cpu().clone() if torch.is_tensor(v) else torch.from_numpy(np.ascontiguousarray(v)).clone()


def hybrid_state_dict(dims: ModelDims, gcn: dict, theta) -> dict:
    """Full HybridSTGCN_LSTM state_dict (reference key order) from the frozen GCN tensors
    (incl. ``base_stgcn.output_layer.*``) and the trainable flat vector / dict."""
    tr = params.unpack(theta, dims, 0) if torch.is_tensor(theta) else theta
    sd = {}
    for name, _ in synth.all_param_specs(dims):
        sd[name] = _t(tr[name]) if name in tr else _t(gcn[name])
    return sd


def adamw_state_dict(dims: ModelDims, m, v, step: int, lr: float, betas=(0.9, 0.999), eps=1e-8,
                     weight_decay=1e-4, initial_lr=None) -> dict:
    """torch.optim.AdamW.state_dict() for param list hybrid.parameters() + koppen.parameters()
    (train_hybrid_maml_v5.py:245-249): state only for the 18 trainable tensors (the others
    never receive a gradient, F2)."""
    names = [n for n, _ in synth.all_param_specs(dims)]
    mm = params.unpack(m, dims, 0)
    vv = params.unpack(v, dims, 0)
    state = {}
    if step > 0:
        for i, n in enumerate(names):
            if n in mm:
                state[i] = {"step": torch.tensor(float(step)), "exp_avg": _t(mm[n]), "exp_avg_sq": _t(vv[n])}
    group = {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay, "amsgrad": False,
             "foreach": None, "maximize": False, "capturable": False, "differentiable": False, "fused": None,
             "decoupled_weight_decay": True,
             "initial_lr": lr if initial_lr is None else initial_lr, "params": list(range(len(names) + 1))}
    return {"state": state, "param_groups": [group]}


def config_dicts(dims: ModelDims, lstm_dropout: float = 0.2):
    return ({"input_channels": dims.input_channels, "hidden_channels": dims.hidden_channels,
             "output_channels": dims.output_channels, "window_size": dims.window_size,
             "forecast_horizon": dims.forecast_horizon},
            {"lstm_hidden_size": dims.lstm_hidden_size, "lstm_num_layers": dims.lstm_num_layers,
             "lstm_dropout": lstm_dropout})


def meta_checkpoint(dims: ModelDims, gcn: dict, theta, koppen_state: dict, m, v, step: int,
                    scheduler_state: dict, epoch: int, best_loss: float, final_loss=None, lr=1e-3,
                    initial_lr=1e-3) -> dict:
    config, hybrid_config = config_dicts(dims)
    total = sum(int(np.prod(s)) for _, s in synth.all_param_specs(dims))
    ck = {
        "hybrid_model_state_dict": hybrid_state_dict(dims, gcn, theta),
        "koppen_embed_state_dict": {k: _t(v_) for k, v_ in koppen_state.items()},
        "meta_optimizer_state_dict": adamw_state_dict(dims, m, v, step, lr, initial_lr=initial_lr),
        "scheduler_state_dict": scheduler_state,
        "epoch": epoch,
    }
    if final_loss is not None:
        ck["final_loss"] = final_loss
    ck.update({"best_loss": best_loss, "model_version": MODEL_VERSION, "total_params": total,
               "config": config, "hybrid_config": hybrid_config})
    return ck


def adapted_checkpoint(dims: ModelDims, gcn: dict, theta, koppen_state: dict, region, region_name: str,
                       stats: dict, val_loss: float, base_model_loss="N/A") -> dict:
    config, hybrid_config = config_dicts(dims)
    total = sum(int(np.prod(s)) for _, s in synth.all_param_specs(dims))
    return {
        "hybrid_model_state_dict": hybrid_state_dict(dims, gcn, theta),
        "koppen_embed_state_dict": {k: _t(v_) for k, v_ in koppen_state.items()},
        "region": region, "region_name": region_name, "climate_type": "Adapted_Region",
        "stats": stats, "config": config, "hybrid_config": hybrid_config, "model_version": MODEL_VERSION,
        "adaptation_type": "v5_regional_adaptation_adaptive", "val_loss": val_loss,
        "base_model_loss": base_model_loss, "total_params": total,
    }


def save(ck: dict, path: str):
    torch.save(ck, path)


def load(path: str, weights_only: bool = True) -> dict:
    """Meta checkpoints load with ``weights_only=True``. Adapted checkpoints carry numpy
    ``stats``; load those only if this code wrote them (``weights_only=False``)."""
    return torch.load(path, map_location="cpu", weights_only=weights_only)


def split_state(dims: ModelDims, sd: dict):
    """hybrid_model_state_dict -> (gcn dict incl. base_stgcn.output_layer, trainable dict)."""
    tr_names = {n for n, _ in synth.trainable_param_specs(dims)}
    gcn = {k: v for k, v in sd.items() if k not in tr_names}
    tr = {k: v for k, v in sd.items() if k in tr_names}
    return gcn, tr


def dims_from_checkpoint(ck: dict, num_nodes: int) -> ModelDims:
    c, h = ck["config"], ck["hybrid_config"]
    return ModelDims(num_nodes=num_nodes, window_size=c["window_size"], input_channels=c["input_channels"],
                     hidden_channels=c["hidden_channels"], lstm_hidden_size=h["lstm_hidden_size"],
                     lstm_num_layers=h["lstm_num_layers"], forecast_horizon=c["forecast_horizon"],
                     output_channels=c["output_channels"])
