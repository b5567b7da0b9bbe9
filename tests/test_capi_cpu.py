"""CPU-only checks of the C ABI library and the host logic (no compute calls)."""
import os
import re

import numpy as np
import pytest
import torch

from oracle import refcpu
from weatherforecast_stgcn_maml_amd import _capi, graph, params, synth
from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2, MamlConfig
from weatherforecast_stgcn_maml_amd.maml import shard_tasks, stream_len_for, window_table

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "smaml.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(smaml_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _capi.lib()
    decl = header_functions()
    assert decl == sorted(_capi.EXPORTS)
    for name in decl:
        assert hasattr(L, name), name
    assert L.smaml_abi_version() == _capi.ABI_VERSION


def test_build_info_reports_every_gemm_family():
    """smaml_build_info (host-only): the product form of each GEMM family of this build
    (0 = f32 MFMA, 1 = bf16x6 fragment split, 2 = bf16x6 staged split)."""
    forms = _capi.product_forms()
    assert set(forms) == {"gcn", "gate", "gate_dual", "bptt", "bptt_dual", "wgrad"}
    assert all(v in (0, 1, 2) for v in forms.values())


@pytest.mark.parametrize("d", [CONFIG1, CONFIG2])
def test_param_layout_matches_state_dict(d):
    lay, total = params.trainable_layout(d)
    specs = synth.trainable_param_specs(d)
    assert [n for n, _, _ in lay] == [n for n, _ in specs]
    prev_end = 0
    for name, shape, off in lay:
        assert off % 64 == 0 and off >= prev_end
        prev_end = off + int(np.prod(shape))
    assert total >= prev_end
    if d == CONFIG2:
        assert params.trainable_count(d) == 606304
        all_params = sum(int(np.prod(s)) for _, s in synth.all_param_specs(d))
        assert all_params == 834752


def test_pack_unpack_roundtrip():
    d = CONFIG1
    P = synth.init_params(0, d)
    t = {k: v for k, v in P.items() if k.startswith(("lstm.", "output_layer."))}
    flat = params.pack(t, d)
    back = params.unpack(flat, d)
    for k, v in t.items():
        assert np.array_equal(back[k].numpy(), v)
    lay, total = params.trainable_layout(d)
    used = np.zeros(total, bool)
    for _, shape, off in lay:
        used[off:off + int(np.prod(shape))] = True
    assert np.all(flat.numpy()[~used] == 0)


@pytest.mark.parametrize("d", [CONFIG1, CONFIG2])
def test_ell_matches_python_restatement_and_pyg_norm(d):
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    ei, n, _ = graph.build_spatial_graph(lats, lons, 4)
    c_cols, c_vals = _capi.graph_ell(ei, n)
    p_cols, p_vals = graph.gcn_ell(ei, n)
    np.testing.assert_array_equal(c_cols, p_cols)
    np.testing.assert_allclose(c_vals, p_vals, rtol=1e-7)
    # the dense t=0 block of PyG's normalised adjacency (oracle) equals the ELL
    x = torch.eye(n)
    dense = refcpu.gcn_conv(x, torch.from_numpy(ei), torch.eye(n), torch.zeros(n)).numpy()
    ell_dense = np.zeros((n, n), np.float32)
    for i in range(n):
        for c, v in zip(c_cols[i], c_vals[i]):
            ell_dense[i, c] += v
    np.testing.assert_allclose(ell_dense, dense, rtol=1e-6, atol=1e-7)


def test_ell_rejects_bad_edges():
    with pytest.raises(_capi.SmamlError):
        _capi.graph_ell(np.array([[0, 1], [1, 5]]), 3)
    star = np.array([[i for i in range(1, 10)], [0] * 9])  # in-degree 9 > 7
    with pytest.raises(_capi.SmamlError):
        _capi.graph_ell(star, 10)


def test_create_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_capi.SmamlError):
        _capi.Context(CONFIG1, 0)


def test_window_table_reference_schedule():
    """Support: the reference's 6 epochs x first 15 support samples at batch 1; query:
    query_ds[0] = sample int(0.75 * min(600, len(dataset))) (train_hybrid_maml_v5.py:97-104,
    162-164), e.g. 450 for a full 600-sample task."""
    from weatherforecast_stgcn_maml_amd.maml import reference_query_start
    cfg = MamlConfig(inner_steps=90, batch=1, order=0, support_samples=15)
    w = window_table(cfg, 2, query_start=reference_query_start(600))
    assert w.shape == (91, 2, 1)
    assert list(w[:, 0, 0][:16]) == list(range(15)) + [0]
    assert w[-1, 0, 0] == 450 and w[-1, 1, 0] == 450
    assert reference_query_start(20) == 15 and reference_query_start(1000) == 450
    w = window_table(cfg, 2, query_start=[7, 9])
    assert list(w[-1, :, 0]) == [7, 9]
    cfg2 = MamlConfig(inner_steps=5, batch=32)
    w2 = window_table(cfg2, 15)
    assert w2[4, 3, 31] == 159 and w2[5, 0, 0] == 160
    # the bench's streams: the reference split puts the query batch right after the support
    n = synth.num_samples(stream_len_for(cfg2, CONFIG2))
    assert reference_query_start(n) == 160 and n - 160 >= 32
    for K, B in [(2, 2), (2, 1), (1, 2), (10, 32)]:
        c = MamlConfig(inner_steps=K, batch=B)
        n = synth.num_samples(stream_len_for(c, CONFIG2))
        assert reference_query_start(n) >= K * B and n - reference_query_start(n) >= B


def test_query_start_never_inside_the_support_samples():
    """a short stream (or S > 450) would put the reference split's query batch inside
    the S support samples; query_starts moves it to S, or raises when the stream is too short."""
    from weatherforecast_stgcn_maml_amd.maml import query_starts, reference_query_start
    cfg = MamlConfig(inner_steps=2, batch=2)  # S = 4
    assert query_starts(cfg, [600, 20, 6]) == [450, 15, 4]   # 20 -> reference split; 6 -> clamped to S
    assert reference_query_start(6) == 4 and reference_query_start(5) == 3
    assert query_starts(cfg, [7]) == [5]
    with pytest.raises(ValueError):
        query_starts(cfg, [5])                               # 4 support + 2 query samples do not fit
    big = MamlConfig(inner_steps=10, batch=60)               # S = 600 > 450: never the reference split
    n = synth.num_samples(stream_len_for(big, CONFIG2))
    assert n >= 660 and query_starts(big, [n]) == [600]
    with pytest.raises(ValueError):
        query_starts(big, [640])
    w = window_table(big, 1, query_start=query_starts(big, [n]))
    assert w[:10].max() < w[10].min()                        # the query batch follows every support sample


def test_shard_tasks_round_robin():
    got = [shard_tasks(15, r, 8) for r in range(8)]
    assert sorted(sum(got, [])) == list(range(15))
    assert [len(g) for g in got] == [2, 2, 2, 2, 2, 2, 2, 1]
    assert shard_tasks(64, 3, 8) == list(range(3, 64, 8))


def test_synth_sample_layout_matches_dataset_contract():
    d = CONFIG1
    f = synth.make_features(0, d.num_nodes, synth.t_total_for(3))
    assert synth.num_samples(f.shape[0]) == 3
    x, y = synth.sample_xy(f, 2)
    assert x.shape == (24 * 25, 24) and y.shape == (8 * 25, 12)
    np.testing.assert_array_equal(x[25 * 3:25 * 4], f[2 + 3])
    np.testing.assert_array_equal(y[25 * 7:25 * 8], f[2 + 24 + 1 + 7, :, :12])
