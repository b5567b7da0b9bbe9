"""k-NN spatial graph (input producer) and the normalised t=0 adjacency.

``build_spatial_graph`` follows ``graphBuilder.py:9-47``: an ``ij`` meshgrid of
(lat, lon), a cKDTree k+1 query, drop the first hit (self), edges ``[node, neighbour]``
(source = node, target = neighbour in PyG's ``source_to_target`` flow). E = k*N, the
graph is not symmetric (border tie-breaking).

``gcn_ell`` restates PyG 2.x ``gcn_norm`` for the t=0 block: self-loops are
added for every row, ``deg = 1 + in-degree`` (counted at the target), ``norm(s->d) =
deg_s^-1/2 deg_d^-1/2``. Rows >= N (t >= 1) have only their self-loop and degree 1, so
their aggregation is the identity; only the first N rows of each sample need the ELL.
"""
from __future__ import annotations

import numpy as np

ELL_WIDTH = 8


def build_spatial_graph(lats, lons, k_neighbors: int = 4):
    from scipy.spatial import cKDTree

    lat_grid, lon_grid = np.meshgrid(np.asarray(lats), np.asarray(lons), indexing="ij")
    pos = np.c_[lat_grid.ravel(), lon_grid.ravel()]
    tree = cKDTree(pos)
    _, nbr = tree.query(pos, k=k_neighbors + 1)
    src = np.repeat(np.arange(len(pos), dtype=np.int64), k_neighbors)
    dst = nbr[:, 1:].reshape(-1).astype(np.int64)
    return np.stack([src, dst]), len(pos), pos


def gcn_ell(edge_index: np.ndarray, num_nodes: int, width: int = ELL_WIDTH):
    """Return ``(cols int32 [N, width], vals float32 [N, width])``: row ``d`` of the
    normalised ``D^-1/2 (A+I) D^-1/2`` restricted to the t=0 block, padded with
    (d, 0.0). Edges in the input are assumed free of self loops (graphBuilder drops
    self); any present are replaced, as PyG's ``add_remaining_self_loops`` does."""
    ei = np.asarray(edge_index, dtype=np.int64)
    src, dst = ei[0], ei[1]
    keep = src != dst
    src, dst = src[keep], dst[keep]
    if src.size and (src.max() >= num_nodes or dst.max() >= num_nodes or src.min() < 0):
        raise ValueError("edge_index references nodes outside [0, num_nodes)")
    deg = np.ones(num_nodes, dtype=np.float64)
    np.add.at(deg, dst, 1.0)
    dinv = np.float32(1.0) / np.sqrt(deg.astype(np.float32))
    cols = np.tile(np.arange(num_nodes, dtype=np.int32)[:, None], (1, width))
    vals = np.zeros((num_nodes, width), dtype=np.float32)
    fill = np.zeros(num_nodes, dtype=np.int64)
    for s, d in zip(src.tolist(), dst.tolist()):
        j = fill[d]
        if j >= width - 1:
            raise ValueError(f"in-degree of node {d} exceeds ELL width {width - 1}")
        cols[d, j] = s
        vals[d, j] = dinv[s] * dinv[d]
        fill[d] += 1
    for d in range(num_nodes):
        cols[d, fill[d]] = d
        vals[d, fill[d]] = dinv[d] * dinv[d]
    return cols, vals
