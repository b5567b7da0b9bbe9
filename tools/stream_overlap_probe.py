"""Probe: do two independent task chains on two HIP streams fill each other's GEMM / epilogue
phase gaps? Second-order config-2 meta-steps (B=32, K=5, all steps kept):
  seq   -- two MetaLearners of 2 tasks each, one after the other on one stream
  conc  -- the same two learners, each on its own stream (kernels may run concurrently)
  one4  -- one MetaLearner of 4 tasks (the launch-size effect alone)
Prints ms per (4-task) meta-step for each."""
import sys
import time

import torch

sys.path.insert(0, ".")
from weatherforecast_stgcn_maml_amd import synth  # noqa: E402
from weatherforecast_stgcn_maml_amd.config import SEED, MamlConfig, ModelDims  # noqa: E402
from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph  # noqa: E402
from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for  # noqa: E402

STEPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d = ModelDims(num_nodes=441)
cfg = MamlConfig(inner_steps=5, batch=32, order=2)
lats, lons = synth.region_grid(n_lat=21, n_lon=21)
ei = build_spatial_graph(lats, lons, 4)[0]
P = synth.init_params(SEED, d)
names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
T_total = stream_len_for(cfg, d)


def learner(ids):
    ml = MetaLearner(d, cfg, {k: v for k, v in P.items() if k not in names}, {k: P[k] for k in names}, ei,
                     device="cuda:0", task_group=None)
    ml.set_tasks([synth.make_features(synth.task_seed(j), d.num_nodes, T_total) for j in ids], task_ids=ids)
    return ml


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / STEPS * 1e3


a, b = learner([0, 1]), learner([2, 3])
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def seq():
    a.meta_step(sync=False)
    b.meta_step(sync=False)


def conc():
    with torch.cuda.stream(s1):
        a.meta_step(sync=False)
    with torch.cuda.stream(s2):
        b.meta_step(sync=False)


print(f"seq  {timed(seq):8.1f} ms", flush=True)
print(f"conc {timed(conc):8.1f} ms", flush=True)
print(f"seq  {timed(seq):8.1f} ms", flush=True)
print(f"conc {timed(conc):8.1f} ms", flush=True)
a.ctx.close()
b.ctx.close()
del a, b
torch.cuda.empty_cache()
c = learner([0, 1, 2, 3])
print(f"one4 {timed(lambda: c.meta_step(sync=False)):8.1f} ms", flush=True)
