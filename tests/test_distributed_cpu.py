"""World-size-2 gloo tests of the multi-GPU logic on CPU: task sharding, the single
meta-gradient all-reduce, and the replicated outer update (bitwise identical on every rank).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from weatherforecast_stgcn_maml_amd import distributed as D

P = 4099
TASKS = 15


def task_grad(j):
    return torch.from_numpy(np.random.default_rng(j).standard_normal(P).astype(np.float32))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle import refcpu

    r, w = D.init_from_env("gloo")
    assert (r, w) == (rank, world) and D.active()
    mine = D.shard_tasks(TASKS, r, w)
    buf = torch.zeros(P + 1)  # MetaLearner's [meta-gradient | query-loss sum]: one collective
    g, q = buf[:P], buf[P:]
    for j in mine:
        g += task_grad(j)
        q += 0.5 * (1.0 + 0.01 * j)
    D.reduce_meta(buf)
    theta = {"p": torch.linspace(-1, 1, P)}
    state = {}
    refcpu.adamw_step(theta, {"p": g}, state, lr=1e-3)
    gathered = [torch.zeros(P) for _ in range(w)]
    dist.all_gather(gathered, theta["p"])
    el = D.max_over_ranks(float(rank + 1), "cpu")
    out_q.put((rank, mine, g.numpy(), float(q), theta["p"].numpy(), [x.numpy() for x in gathered], el))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_rank_meta_reduction_and_replicated_update(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assigned = sorted(sum([r[1] for r in res], []))
    assert assigned == list(range(TASKS))
    full = sum(task_grad(j) for j in range(TASKS))
    for r in res:
        np.testing.assert_allclose(r[2], full.numpy(), rtol=1e-5, atol=1e-5)
        assert abs(r[3] - sum(0.5 * (1.0 + 0.01 * j) for j in range(TASKS))) < 1e-5
        assert r[6] == float(world)
    # every rank holds bit-identical parameters after the replicated outer step
    for r in res:
        for other in r[5]:
            assert np.array_equal(other, res[0][4])
