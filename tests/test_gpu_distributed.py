"""Multi-rank MetaLearner on the GPU path (train_hybrid_maml_v5.py:144-184):
tasks sharded round-robin over ranks, the meta-step's ONE all-reduce of [meta-gradient |
query-loss sum], then the replicated clip + AdamW. Two ranks share the test box's one GPU over
gloo (RCCL needs one GPU per rank; the driver's 8-GPU bench runs the same code over RCCL). Each
rank is a freshly spawned process (never an exec of a process that touched the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, tasks, out_q, config="cfg1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist

    from weatherforecast_stgcn_maml_amd import synth
    from weatherforecast_stgcn_maml_amd.config import CONFIG1, CONFIG2, MamlConfig
    from weatherforecast_stgcn_maml_amd.distributed import init_from_env, shard_tasks
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    torch.cuda.set_device(0)
    if world > 1:
        init_from_env("gloo")
    d = CONFIG1 if config == "cfg1" else CONFIG2
    cfg = MamlConfig(inner_steps=2, batch=2 if config == "cfg1" else 4, order=2)
    P = synth.init_params(31, d, gcn_bias_scale=0.1)
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    ei = build_spatial_graph(lats, lons, 4)[0]
    mine = shard_tasks(tasks, rank, world)
    feats = [synth.make_features(synth.task_seed(j), d.num_nodes, stream_len_for(cfg, d)) for j in mine]
    ml = MetaLearner(d, cfg, {k: v for k, v in P.items() if k not in names}, {k: P[k] for k in names}, ei,
                     device="cuda:0")
    ml.set_tasks(feats, task_ids=mine)
    meta_losses, mg1 = [], None
    for i in range(STEPS):
        meta_losses.append(ml.meta_step().meta_loss)
        if i == 0:  # the first step's all-reduced meta-gradient (both sides at the same theta)
            mg1 = ml.meta_grad.cpu().numpy().copy()
    out_q.put((rank, mine, ml.theta.cpu().numpy(), meta_losses, mg1))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _run(world, tasks, config="cfg1"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, tasks, q, config)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _comm_main(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from weatherforecast_stgcn_maml_amd import _capi
    from weatherforecast_stgcn_maml_amd.config import CONFIG1
    from weatherforecast_stgcn_maml_amd.distributed import capi_comm_check

    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    ctx = _capi.Context(CONFIG1, rank)
    out_q.put((rank, capi_comm_check(ctx, 1 << 20, iters=3)))
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_capi_rccl_communicator(world):
    """The C ABI's own RCCL communicator (smaml_comm_unique_id / init / allreduce / destroy,
    include/smaml.h) through distributed.capi_comm_check, the collective a non-torch host binds
    for the outer step (train_hybrid_maml_v5.py:174-179); bench.py runs the same check at every
    N>1. RCCL rejects two ranks on one device ("Duplicate GPU detected"), so world 2 needs a box
    with two GPUs; world 1 runs the same id exchange, init, all-reduce and destroy."""
    import torch
    n = torch.cuda.device_count()
    if n < world:
        pytest.skip(f"{n} GPU(s) visible: RCCL needs one GPU per rank")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, r in res:
        assert r["status"] == "ok", r
        assert r["world"] == world and r["elements"] == 1 << 20 and r["allreduce_ms"] > 0


@pytest.mark.parametrize("tasks", [4, 1])
def test_two_rank_meta_learner_matches_one_rank(tasks):
    """tasks = 1: rank 1 holds no task; it still joins the one all-reduce with zeros and takes
    the replicated AdamW step (maml.py Z == 0 path), so both ranks end on the 1-rank theta."""
    one = _run(1, tasks)[0]
    two = _run(2, tasks)
    assert sorted(two[0][1] + two[1][1]) == list(range(tasks))
    assert bool(two[1][1]) == (tasks > 1)
    # replicated outer step on the all-reduced meta-gradient: bitwise identical on every rank
    assert np.array_equal(two[0][2], two[1][2])
    assert two[0][3] == two[1][3]  # meta_loss (all-reduced query-loss sum) identical too
    # and the 1-rank result up to the summation order of the task meta-gradients
    err = np.linalg.norm(two[0][2] - one[2]) / np.linalg.norm(one[2])
    assert err <= 1e-6, err
    if tasks == 1:  # one task: the same sum on both sides, bitwise
        assert np.array_equal(two[0][2], one[2])
    assert not np.array_equal(one[2], np.zeros_like(one[2]))
    np.testing.assert_allclose(two[0][3], one[3], rtol=1e-6)


def test_two_rank_meta_learner_cfg2_shapes():
    """The same sharding at BASELINE config-2 shapes (N=441, Hc=256, LSTM 4x128; B=4, K=2, second order,
    3 tasks: rank 0 holds two, rank 1 one): the all-reduced meta-gradient equals the one-rank one up to
    the summation order of the task terms (<= 1e-6 rel-L2), and the replicated AdamW leaves theta and the
    meta-loss bitwise identical on both ranks (train_hybrid_maml_v5.py:144-184)."""
    one = _run(1, 3, "cfg2")[0]
    two = _run(2, 3, "cfg2")
    assert sorted(two[0][1] + two[1][1]) == [0, 1, 2] and len(two[0][1]) == 2
    assert np.array_equal(two[0][2], two[1][2]) and two[0][3] == two[1][3]
    assert np.array_equal(two[0][4], two[1][4])
    err = np.linalg.norm(two[0][4] - one[4]) / np.linalg.norm(one[4])
    assert err <= 1e-6, err
    np.testing.assert_allclose(two[0][3][0], one[3][0], rtol=1e-6)  # (step 1: same theta on both sides)
