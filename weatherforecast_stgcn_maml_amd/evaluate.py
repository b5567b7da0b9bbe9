"""Regional evaluation: the metric path of ``validate_hybrid_v5.validateAdapted``
(validate_hybrid_v5.py:189-237, 337-358) on the HIP forward.

The reference runs a no-grad forward on the first ``min(3, len(dataset))`` windows, averages the
predictions and the targets over those samples, reshapes BOTH as ``[Hf, N, 12]`` (the prediction
rows are ``[node][horizon]``-ordered, so this is the same F4 pairing the training loss uses: kept,
not fixed), averages over nodes, denormalises the first six variables with the adaptation
checkpoint's ``stats`` and reports per-variable MSE / MAE over the forecast steps plus their
average without ``sp``. Plots and the NetCDF loading (:137-170, :240-335) are out of scope.

The forward of all samples is one batched ``smaml_forward`` launch sequence; the sample / node
averages run on the device, the 6 x Hf denormalised metrics on the host (as the reference's
numpy does).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from . import _capi

# validate_hybrid_v5.py:19-32
VAR_NAMES = ["u10", "v10", "t2m", "d2m", "sp", "tp", "u100", "v100", "str", "hcc", "lcc", "e"]


def regional_metrics(y_pred_avg: np.ndarray, y_true_avg: np.ndarray, stats, forecast_horizon: int,
                     num_nodes: int) -> Dict:
    """validate_hybrid_v5.py:224-237,337-358 from the sample-averaged prediction / target
    ``[N*Hf, 12]`` arrays: reshape ``[Hf, N, 12]``, node mean, denormalise, MSE / MAE."""
    mean = np.array(stats["mean"]) if isinstance(stats, dict) else np.asarray(stats[0])
    std = np.array(stats["std"]) if isinstance(stats, dict) else np.asarray(stats[1])
    yt = np.asarray(y_true_avg).reshape(forecast_horizon, num_nodes, 12).mean(axis=1)
    yp = np.asarray(y_pred_avg).reshape(forecast_horizon, num_nodes, 12).mean(axis=1)
    return _metrics(yp, yt, mean, std)


def _metrics(yp, yt, mean, std):
    results, total, count = {}, 0.0, 0
    for v, name in enumerate(VAR_NAMES[:6]):
        if v < yt.shape[1]:
            t = yt[:, v] * std[v] + mean[v]
            p = yp[:, v] * std[v] + mean[v]
            mse = np.mean((p - t) ** 2)
            results[name] = {"mse": mse, "mae": np.mean(np.abs(p - t))}
            if name != "sp":  # surface pressure is excluded from the average (:352-355)
                total += mse
                count += 1
    results["average_mse"] = total / count if count else 0
    return results


def evaluate_regional(model, features, edge_index, stats, num_samples: int = 3) -> Dict:
    """``model``: the drop-in ``HybridSTGCN_LSTM`` (its weights); ``features``: the region's
    normalised ``[T_total, N, 24]`` stream (a tensor on the HIP device or a numpy array);
    ``stats``: ``{"mean": [12], "std": [12]}`` of the adaptation checkpoint. Returns the
    reference's results dict (per-variable ``{"mse", "mae"}`` and ``"average_mse"``)."""
    dev = next(model.parameters()).device
    if dev.type != "cuda":
        raise _capi.SmamlError(-1, "evaluate_regional runs on a HIP device only")
    f = features if torch.is_tensor(features) else torch.from_numpy(np.ascontiguousarray(features))
    f = f.to(dev, torch.float32).contiguous()
    T = model.base_stgcn.window_size
    Hf, C = model.forecast_horizon, model.out_channels
    N = f.shape[1]
    n = min(num_samples, max(0, f.shape[0] - T - Hf))  # len(WeatherGraphDataset) (dataset.py:25)
    if n == 0:
        return {"average_mse": float("inf")}
    ei = edge_index if torch.is_tensor(edge_index) else torch.from_numpy(np.asarray(edge_index))
    xs = [f[i:i + T].reshape(T * N, -1) for i in range(n)]  # windows are views of the stream
    ctx, dims, theta = model._prepare(xs[0], ei)
    pred = torch.empty(n, N * Hf, C, device=dev)
    with torch.no_grad():
        ctx.forward(_capi.stream_ptr(torch), theta, xs, pred)
        y_pred = pred.mean(0)
        y_true = torch.stack([f[i + T + 1:i + T + 1 + Hf, :, :12].reshape(Hf * N, 12) for i in range(n)]).mean(0)
        yp = y_pred.view(Hf, N, C).mean(1).double().cpu().numpy()
        yt = y_true.view(Hf, N, 12).mean(1).double().cpu().numpy()
    mean = np.array(stats["mean"]) if isinstance(stats, dict) else np.asarray(stats[0])
    std = np.array(stats["std"]) if isinstance(stats, dict) else np.asarray(stats[1])
    return _metrics(yp, yt, mean, std)
