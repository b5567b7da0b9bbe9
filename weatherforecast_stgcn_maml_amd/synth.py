"""Portable synthetic ERA5-shaped inputs and reference-distribution weights.

Everything here is driven by numpy ``default_rng`` (PCG64) seeds so that the GPU box can
regenerate exactly the arrays the golden fixtures were made from.

Feature layout follows ``featurePreprocessor.prepare_model_input``
(``featurePreprocessor.py:170-177``): channels 0-11 weather (z-scored), 12-15 time
embeddings (``embed_utils.add_time_embeddings``, ``embed_utils.py:10-27``), 16-23 the
Köppen embedding broadcast over time and nodes. The stream is ``[T_total, N, 24]``;
sample ``i`` of a task is the window starting at time ``i`` (``dataset.py:25,30-48``).
"""
from __future__ import annotations

import numpy as np

from .config import ModelDims, WINDOW_SIZE, FORECAST_HORIZON


def region_grid(lat_max: float = 23.0, lon_min: float = 75.0, n_lat: int = 21, n_lon: int = 21,
                step: float = 0.25):
    """ERA5-style coordinates: latitude descending, longitude ascending (0.25 deg)."""
    lats = lat_max - step * np.arange(n_lat, dtype=np.float64)
    lons = lon_min + step * np.arange(n_lon, dtype=np.float64)
    return lats, lons


def grid_shape(num_nodes: int):
    side = int(round(num_nodes ** 0.5))
    if side * side != num_nodes:
        raise ValueError(f"num_nodes={num_nodes} is not a square grid")
    return side, side


def make_features(seed: int, num_nodes: int, t_total: int, ar: float = 0.0,
                  start_hour: int = 0) -> np.ndarray:
    """``[t_total, num_nodes, 24]`` float32 feature stream for one task/region."""
    rng = np.random.default_rng(seed)
    weather = rng.standard_normal((t_total, num_nodes, 12), dtype=np.float32)
    if ar:
        a = np.float32(ar)
        s = np.float32(np.sqrt(1.0 - ar * ar))
        for t in range(1, t_total):
            weather[t] = a * weather[t - 1] + s * weather[t]
    hours = start_hour + np.arange(t_total, dtype=np.float64)
    day_of_year = 1.0 + np.floor(hours / 24.0) % 365
    time_of_day = hours % 24.0
    yp = 2 * np.pi * day_of_year / 365.25
    dp = 2 * np.pi * time_of_day / 24.0
    tf = np.stack([np.sin(yp), np.cos(yp), np.sin(dp), np.cos(dp)], axis=-1).astype(np.float32)
    koppen = rng.standard_normal(8).astype(np.float32)
    feats = np.empty((t_total, num_nodes, 24), dtype=np.float32)
    feats[:, :, :12] = weather
    feats[:, :, 12:16] = tf[:, None, :]
    feats[:, :, 16:24] = koppen[None, None, :]
    return feats


def num_samples(t_total: int, window: int = WINDOW_SIZE, horizon: int = FORECAST_HORIZON) -> int:
    """``len(WeatherGraphDataset)`` (dataset.py:25)."""
    return max(0, t_total - window - horizon)


def t_total_for(samples: int, window: int = WINDOW_SIZE, horizon: int = FORECAST_HORIZON) -> int:
    return samples + window + horizon


def sample_xy(features: np.ndarray, i: int, window: int = WINDOW_SIZE,
              horizon: int = FORECAST_HORIZON):
    """``WeatherGraphDataset.__getitem__`` restated (dataset.py:30-48), F5 included:
    ``x = features[i:i+W].reshape(W*N, 24)`` (time-major rows) and
    ``y[h*N + n] = features[i+W+1+h, n, :12]`` (horizon-major rows, targets skip t+0)."""
    n = features.shape[1]
    x = features[i:i + window].reshape(window * n, -1)
    y = features[i + window + 1:i + window + 1 + horizon, :, :12].reshape(horizon * n, 12)
    return x, y


# --------------------------------------------------------------------------------------
# Parameters (state_dict order of hybrid_model.HybridSTGCN_LSTM)
# --------------------------------------------------------------------------------------

def gcn_param_specs(d: ModelDims):
    specs = []
    cin = d.input_channels
    for k in range(1, 5):
        specs.append((f"base_stgcn.conv{k}.bias", (d.hidden_channels,)))
        specs.append((f"base_stgcn.conv{k}.lin.weight", (d.hidden_channels, cin)))
        cin = d.hidden_channels
    specs.append(("base_stgcn.output_layer.weight", (d.head_out, d.hidden_channels)))
    specs.append(("base_stgcn.output_layer.bias", (d.head_out,)))
    return specs


def trainable_param_specs(d: ModelDims):
    """LSTM + head: the 18 (for 4 layers) tensors that receive gradients (F2)."""
    specs = []
    H = d.lstm_hidden_size
    for l in range(d.lstm_num_layers):
        cin = d.hidden_channels if l == 0 else H
        specs.append((f"lstm.weight_ih_l{l}", (4 * H, cin)))
        specs.append((f"lstm.weight_hh_l{l}", (4 * H, H)))
        specs.append((f"lstm.bias_ih_l{l}", (4 * H,)))
        specs.append((f"lstm.bias_hh_l{l}", (4 * H,)))
    specs.append(("output_layer.weight", (d.head_out, H)))
    specs.append(("output_layer.bias", (d.head_out,)))
    return specs


def all_param_specs(d: ModelDims):
    return gcn_param_specs(d) + trainable_param_specs(d)


def init_params(seed: int, d: ModelDims, gcn_bias_scale: float = 0.0) -> dict:
    """Weights drawn with the reference's init distributions (PyG glorot for GCN lin,
    zeros for GCN bias unless ``gcn_bias_scale``; ``nn.LSTM`` U(+-1/sqrt(H));
    ``nn.Linear`` U(+-1/sqrt(fan_in)))."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in all_param_specs(d):
        if ".lin.weight" in name:
            a = np.sqrt(6.0 / (shape[0] + shape[1]))
            v = rng.uniform(-a, a, size=shape)
        elif name.startswith("base_stgcn.conv"):
            v = (rng.uniform(-gcn_bias_scale, gcn_bias_scale, size=shape)
                 if gcn_bias_scale else np.zeros(shape))
        elif name.startswith("lstm."):
            a = 1.0 / np.sqrt(d.lstm_hidden_size)
            v = rng.uniform(-a, a, size=shape)
        else:  # Linear layers
            fan_in = d.hidden_channels if name.startswith("base_stgcn") else d.lstm_hidden_size
            a = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-a, a, size=shape)
        out[name] = np.ascontiguousarray(v, dtype=np.float32)
    return out


def task_seed(j: int) -> int:
    """task j uses seed 1000+j."""
    return 1000 + j
