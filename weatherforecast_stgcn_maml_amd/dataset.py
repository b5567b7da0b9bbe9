"""Drop-in for the reference ``dataset.py`` (``WeatherGraphDataset``), as a layout contract.

``features`` is a ``[T_total, N, 24]`` stream (torch tensor, may live in HBM); sample ``idx``
is the window ``features[i-W:i]`` with targets ``features[i+1..i+H, :, :12]`` where
``i = valid_indices[idx]`` (dataset.py:25,30-48; F5). Items are ``GraphSample`` objects with
``.x [W*N, 24]`` (time-major rows), ``.edge_index``, ``.y [H*N, 12]`` (horizon-major rows)
and ``.to(device)`` like PyG's ``Data``. The MAML driver never materialises items: it hands
the library window starts (``window_start``) into the resident stream.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch.utils.data import Dataset


@dataclass
class GraphSample:
    x: torch.Tensor
    edge_index: torch.Tensor
    y: torch.Tensor

    def to(self, device):
        return GraphSample(self.x.to(device), self.edge_index.to(device), self.y.to(device))


class WeatherGraphDataset(Dataset):
    def __init__(self, features, edge_index, window_size=6, forecast_horizon=1):
        self.features = features
        self.edge_index = edge_index
        self.window_size = window_size
        self.forecast_horizon = forecast_horizon
        self.num_weather_vars = 12
        self.num_nodes = features.shape[1]
        self.valid_indices = range(window_size, len(features) - forecast_horizon)

    def __len__(self):
        return len(self.valid_indices)

    def window_start(self, idx: int) -> int:
        """Stream index of the first time step of sample ``idx``'s window."""
        return self.valid_indices[idx] - self.window_size

    def __getitem__(self, idx):
        i = self.valid_indices[idx]
        W, H, N = self.window_size, self.forecast_horizon, self.num_nodes
        x = self.features[i - W:i].reshape(W * N, -1)
        y = self.features[i + 1:i + H + 1, :, :self.num_weather_vars].reshape(H * N, self.num_weather_vars)
        return GraphSample(x.clone(), self.edge_index, y.clone())


def resolve_windows(ds):
    """(stream tensor, [window starts]) of a WeatherGraphDataset or a Subset of one."""
    indices = None
    while hasattr(ds, "indices") and hasattr(ds, "dataset"):
        sub = list(ds.indices)
        indices = sub if indices is None else [sub[i] for i in indices]
        ds = ds.dataset
    if not hasattr(ds, "valid_indices"):
        raise TypeError("expected a WeatherGraphDataset (or Subset of one)")
    if indices is None:
        indices = list(range(len(ds)))
    return ds.features, [ds.valid_indices[i] - ds.window_size for i in indices], ds
