"""Benchmark: MAML meta-steps/sec on BASELINE config 2 (15 tasks x B=32 x T=24 x N=441,
Hc=256, LSTM 4x128, K=5 inner steps) on 1..8 MI355X, plus the reference's CPU path.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 launched by
torch.distributed.run (one rank per GPU, RCCL). Prints ONE JSON line on rank 0.

One "step" = one meta-step over the 15-task meta-batch: every task runs K inner steps of
B samples (GCN x4 fwd, LSTM fwd, head + loss, BPTT, clip + SGD) and one B-sample query
batch (+ backward for the meta-gradient), then one RCCL all-reduce of the 606,304-float
meta-gradient and a replicated clip + AdamW. Tasks are sharded round-robin over ranks:
the meta-batch is fixed, so scaling is "strong". Inputs are synthetic ERA5-shaped
feature streams (portable numpy seeds 1000+j) resident in HBM before the timed region;
weights are random-init with the reference's distributions.

At N=1, after the headline timed region (never inside it), the same line also carries
BASELINE config 4 (``adaptation``: regional fine-tuning, ms per batch-1 sample-step) and one
rank's share of config 5 (``config5_rank_share``: 8 of the 64 stress tasks, ms per meta-step).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec)
PEAK_BF16_MFMA_TFLOPS = 16 * PEAK_FP32_MFMA_TFLOPS  # dense BF16 MFMA = 16x the f32 MFMA rate (2516.8 TF)
# f32-accurate products as six bf16 piece products (gemm_core.h mfma_x6): 2516.8 / 6 = 419.5 TF of f32 work
PEAK_X6_TFLOPS = PEAK_BF16_MFMA_TFLOPS / 6
PEAK_HBM_GBS = 8000.0
# bound on the N>1 C-ABI RCCL check after the timed region (its init alone waits up to 60 s)
CAPI_COMM_WATCHDOG_S = 150.0
# timing category -> GEMM family of smaml_build_info (product form of its contraction)
CAT_FAMILY = {"gcn_layer": "gcn", "xg_proj": "gate", "lstm_fwd_step": "gate", "lstm_fwd_dual": "gate_dual", "lstm_bwd_step": "bptt",
              "lstm_bwd_dual": "bptt_dual", "wgrad": "wgrad", "head_dh": "bptt", "head_loss": "bptt"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--tasks", type=int, default=15)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--inner-steps", type=int, default=5)
    p.add_argument("--nodes", type=int, default=441)
    p.add_argument("--order", type=int, default=2, help="2 = second-order MAML (BASELINE config 2)")
    p.add_argument("--cpu-sample-steps", type=int, default=6,
                   help="reference-port CPU sample-steps to time (0 = skip)")
    p.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP-event timing")
    p.add_argument("--config", type=int, default=2, choices=(2, 5),
                   help="5 = BASELINE stress config: 64 tasks, N=1024 (32x32), Hc=512, LSTM 4x128, K=10, "
                        "second order (flags given explicitly still win, e.g. --tasks 8 = one rank's share at 8 GPUs)")
    p.add_argument("--hidden-channels", type=int, default=None)
    p.add_argument("--dropout", type=float, nargs=2, default=(0.0, 0.0), metavar=("P_GCN", "P_LSTM"),
                   help="train-mode dropout (the reference trains at 0.2 0.2; 0 0 = the parity setting)")
    p.add_argument("--adapt-epochs", type=int, default=2,
                   help="after the timed region (N=1 only): BASELINE config-4 adaptation epochs to time and "
                        "report under 'adaptation' (0 = skip)")
    p.add_argument("--cfg5-share-tasks", type=int, default=8,
                   help="after the timed region (N=1, config 2 only): time one second-order meta-step of this "
                        "many BASELINE config-5 tasks (8 = one rank's share of the 64 tasks at 8 GPUs) and report "
                        "it under 'config5_rank_share' (0 = skip)")
    p.add_argument("--task-group", default="auto",
                   help="tasks per pass of the C driver: an int, 'all', or 'auto' (default: groups small "
                        "enough that every inner step's primal stays resident for the second-order sweep)")
    args = p.parse_args()
    args.task_group = None if args.task_group == "all" else args.task_group if args.task_group == "auto" \
        else int(args.task_group)
    if args.config == 5:
        given = {a.split("=")[0] for a in sys.argv[1:] if a.startswith("--")}
        for flag, key, val in (("--tasks", "tasks", 64), ("--nodes", "nodes", 1024), ("--inner-steps", "inner_steps", 10),
                               ("--hidden-channels", "hidden_channels", 512), ("--cpu-sample-steps", "cpu_sample_steps", 0)):
            if flag not in given:
                setattr(args, key, val)
    return args


def algorithmic_flops(d, tasks, K, B, order):
    """SURVEY §8(d) convention: per-sample FO step = GCN + LSTM_fwd + head + bwd."""
    T, N, Cin, Hc, H, L = d.window_size, d.num_nodes, d.input_channels, d.hidden_channels, d.lstm_hidden_size, d.lstm_num_layers
    HfC = d.forecast_horizon * d.output_channels
    gcn = 2 * T * N * (Cin * Hc + 3 * Hc * Hc)
    lstm = 2 * T * N * 4 * H * (Hc + H) + 2 * T * N * 4 * H * 2 * H * (L - 1)
    head = 2 * N * H * HfC
    bwd = lstm + (lstm - 2 * T * N * 4 * H * Hc) + 2 * head
    per = gcn + lstm + head + bwd
    fo = tasks * (K + 1) * B * per
    if order == 2:
        return fo + tasks * K * B * 2 * (lstm + head + bwd)
    return fo


def progress(msg):
    """Progress on stderr (the driver reads only the JSON line on stdout)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cgroup_cpus():
    """CPUs the process's cgroup quota grants (cgroup v2 cpu.max or v1 cfs quota), or None."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def cpu_threads():
    """(threads used, os.cpu_count(), CPUs this process may run on). The port is timed with one
    thread per CPU the process can actually use: os.cpu_count() capped by the affinity mask and the
    cgroup CPU quota (on the GPU box os.cpu_count() reports the whole machine, 256, while the quota
    grants 16: 256 threads on 16 CPUs oversubscribe and stall)."""
    n_os = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = n_os
    quota = cgroup_cpus()
    usable = min(n_os, n_aff, quota or n_os)
    return max(1, usable), n_os, min(n_aff, quota or n_aff)


def cpu_baseline(d, n_steps, P, ei, feats):
    """Reference CPU path restated op for op (oracle.refcpu.ReferencePort: per-node nn.LSTM
    loop, batch 1, MKLDNN), timed on this host's cores over a bounded sample. Returns
    (seconds per sample-step, threads used, os.cpu_count(), affinity CPUs)."""
    import torch
    from oracle import refcpu
    from weatherforecast_stgcn_maml_amd import synth

    threads, n_os, n_aff = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        port = refcpu.ReferencePort(P, d, ei)
        x, y = synth.sample_xy(feats, 0)
        x = torch.from_numpy(np.ascontiguousarray(x))
        y = torch.from_numpy(np.ascontiguousarray(y))
        port.step(x, y)  # warm
        t0 = time.perf_counter()
        for i in range(n_steps):
            xi, yi = synth.sample_xy(feats, i % 8)
            port.step(torch.from_numpy(np.ascontiguousarray(xi)), torch.from_numpy(np.ascontiguousarray(yi)))
            progress(f"cpu baseline sample-step {i + 1}/{n_steps} ({threads} threads)")
        t = (time.perf_counter() - t0) / n_steps
        used = torch.get_num_threads()
    finally:
        torch.set_num_threads(prev)
    return t, used, n_os, n_aff


def adaptation_bench(d, P, ei, epochs=2, max_samples=1200, region="Amazon", breakdown_steps=96, warmup=True):
    """BASELINE config 4 (regional adaptation, adapt_hybrid_v5.py:186-208): epochs of shuffled batch-1
    train steps (fwd + bwd + clip + Adam(L2)) of the pretrained init on one N=441 region, each epoch
    one smaml_adapt_steps call on a fresh context (cold per-window GCN feature cache: epoch 1 also
    computes every window's GCN features, later epochs reuse them, F2). The context's workspace and
    cache are allocated before the first epoch (smaml_adapt_prepare, reported as setup_ms), as
    adapt.adapt does; each epoch's phases (reserve / cache alloc / cache fill / steps) are reported. Returns the per-epoch times
    and a per-category kernel breakdown of ``breakdown_steps`` warm steps timed with HIP events in a
    separate pass (the events add launch overhead, so those steps are not the timed value)."""
    import torch

    from weatherforecast_stgcn_maml_amd import _capi, adapt, params, synth

    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    gcn = {k: v for k, v in P.items() if k not in names}
    theta = {k: P[k] for k in names}
    T_total = max_samples + d.window_size + d.forecast_horizon
    feats = synth.make_features(synth.task_seed(0), d.num_nodes, T_total)
    dev = torch.device("cuda", torch.cuda.current_device())
    n_max = min(max_samples, synth.num_samples(T_total, d.window_size, d.forecast_horizon))
    n_train = int(0.8 * n_max)
    lr, wd = adapt.climate_optimizer_config(region, 0.0006)
    stream_t = torch.from_numpy(np.ascontiguousarray(feats)).to(dev)
    stream = _capi.stream_ptr(torch)
    rng = np.random.default_rng(1234)  # shuffle orders (the reference's DataLoader draws its own)

    def run(n_epochs, steps=None, timing=False):
        ctx = _capi.Context(d, dev.index or 0)
        ts = time.perf_counter()
        phases = []
        ctx.set_graph(ei)
        gflat = params.pack(gcn, d, which=1, device=dev)
        ctx.set_gcn_params(gflat)
        th = params.pack(theta, d, which=0, device=dev)
        ctx.set_tasks([stream_t])
        ctx.set_task_ids([0])
        m, v = torch.zeros_like(th), torch.zeros_like(th)
        losses = torch.empty(n_train, device=dev)
        lr_dev = torch.full((n_train,), lr, device=dev, dtype=torch.float32)
        # set-up (as adapt.adapt does before its epochs): workspace + per-window feature cache allocated
        # and touched here, so a driver-side clear of released VRAM cannot land in the first epoch
        ctx.adapt_prepare(stream, 1)
        prep = ctx.adapt_phases()  # (its reserve / cache-allocation phases)
        ctx.set_option("adapt_phase_sync", 1)  # phase times below include GPU time (2 syncs per epoch)
        torch.cuda.synchronize()
        setup_ms = (time.perf_counter() - ts) * 1e3
        phases.append({"prepare_" + k: v for k, v in prep.items() if k in ("reserve_ms", "cache_alloc_ms")})
        per_epoch, step, kern = [], 0, None
        for e in range(n_epochs):
            order = rng.permutation(n_train).astype(np.int32)[:steps or n_train]
            if timing and e == n_epochs - 1:
                ctx.timing_collect()
                ctx.timing(True)
            t0 = time.perf_counter()
            ctx.adapt_steps(stream, th, m, v, step, order.reshape(-1, 1), lr_dev, (0.9, 0.999), 1e-8, wd,
                            adapt.MAX_GRAD_NORM, losses)
            torch.cuda.synchronize()
            per_epoch.append(time.perf_counter() - t0)
            phases.append(ctx.adapt_phases())
            step += len(order)
        if timing:
            ctx.timing(False)
            kern = ctx.timing_collect()
        loss = float(losses[:len(order)].double().mean().item())
        ctx.close()
        return per_epoch, loss, kern, setup_ms, phases

    if warmup:
        run(1, steps=64)  # module load, first touch of a workspace
    per_epoch, loss, _, setup_ms, phases = run(epochs)
    assert np.isfinite(loss), loss
    _, _, kern, _, _ = run(2, steps=breakdown_steps, timing=True)  # epoch 1 fills the cache for the timed steps
    later = per_epoch[1:] or per_epoch
    out = {
        "metric": "regional adaptation ms per later-epoch sample-step (batch-1 fwd+bwd+clip+Adam, N=441, T=24)",
        "value": float(np.mean(later)) / n_train * 1e3,
        "unit": "ms/sample-step",
        "higher_is_better": False,
        "first_epoch_ms": per_epoch[0] * 1e3,
        "later_epoch_ms": float(np.mean(later)) * 1e3,
        "setup_ms": setup_ms,
        "setup_phases_ms": {k: round(v, 3) for k, v in phases[0].items()},
        "epoch_phases_ms": [{k: round(v, 3) for k, v in ph.items()} for ph in phases[1:]],
        "phases_note": "host-timed phases of each smaml_adapt_steps call (smaml_adapt_phases, option "
                       "adapt_phase_sync: fill and steps end with a stream sync); setup_ms = context set-up "
                       "incl. smaml_adapt_prepare (workspace reserve + feature-cache allocation, each touched "
                       "and synced: setup_phases_ms), outside the epochs. Round 5's ~6 s first-epoch stall on "
                       "some boxes was this allocation after the headline run released its ~250 GB",
        "sample_steps_per_s": n_train / float(np.mean(later)),
        "train_loss": loss,
        "config": {"workload": f"BASELINE config 4: {epochs}-epoch adaptation (adapt_hybrid_v5), epochs of {n_train} "
                               f"shuffled batch-1 train steps, N={d.num_nodes}, Hc={d.hidden_channels}, LSTM "
                               f"{d.lstm_num_layers}x{d.lstm_hidden_size}, Adam(L2) lr {lr:g} wd {wd:g} ({region}); "
                               f"GCN features computed once per window (frozen GCN, F2)",
                   "epochs": epochs, "train_samples": n_train},
    }
    if kern:
        out["kernels_us_per_sample_step"] = {k: v["ms"] * 1e3 / breakdown_steps for k, v in kern.items()
                                             if v["launches"] > 0}
        out["launches_per_sample_step"] = {k: v["launches"] / breakdown_steps for k, v in kern.items()
                                           if v["launches"] > 0}
    return out, feats


def config5_share_bench(tasks, steps=1, warmup=1, timing=True):
    """BASELINE config 5 (stress: 64 tasks, N=1024 (32x32 grid), Hc=512, LSTM 4x128, K=10, second
    order), the share one rank holds when the driver's 8-GPU run shards the 64 tasks round-robin:
    ``tasks`` tasks on this GPU, ``warmup`` untimed + ``steps`` timed meta-steps on a fresh
    MetaLearner, after (never inside) the headline timed region. The 8-GPU meta-step is this share
    plus one all-reduce of the 606,304-float meta-gradient."""
    import torch

    from weatherforecast_stgcn_maml_amd import synth
    from weatherforecast_stgcn_maml_amd.config import SEED, MamlConfig, ModelDims
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, stream_len_for

    d = ModelDims(num_nodes=1024, hidden_channels=512)
    cfg = MamlConfig(inner_steps=10, batch=32, order=2)
    lats, lons = synth.region_grid(n_lat=32, n_lon=32)
    ei, _, _ = build_spatial_graph(lats, lons, 4)
    P = synth.init_params(SEED, d)
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    T_total = stream_len_for(cfg, d)
    ids = list(range(tasks))
    feats = [synth.make_features(synth.task_seed(j), d.num_nodes, T_total) for j in ids]
    ml = MetaLearner(d, cfg, {k: v for k, v in P.items() if k not in names}, {k: P[k] for k in names},
                     ei, device=f"cuda:{torch.cuda.current_device()}", dropout_seed=SEED)
    ml.set_tasks(feats, task_ids=ids)
    for _ in range(warmup):
        ml.meta_step(sync=False)
    if timing:
        ml.ctx.timing_collect()  # drop warmup records
        ml.ctx.timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = None
    for _ in range(steps):
        res = ml.meta_step(sync=False)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern = None
    if timing:
        ml.ctx.timing(False)
        kern = ml.ctx.timing_collect()
    qmse = float(res.losses[-1].sum().item()) / tasks
    kept = ml.ctx.so_kept_steps()
    groups = len(ml._groups)
    ml.ctx.close()
    del ml
    torch.cuda.empty_cache()
    assert np.isfinite(qmse), qmse
    flops = algorithmic_flops(d, tasks, cfg.inner_steps, cfg.batch, cfg.order)
    ms = elapsed / steps * 1e3
    out = {
        "metric": "config-5 rank share: ms per second-order meta-step of one rank's tasks",
        "value": ms, "unit": "ms/meta-step", "higher_is_better": False, "steps": steps, "warmup": warmup,
        "meta_step_tflop": flops / 1e12,
        "achieved_tflops_whole_step": flops / (elapsed / steps) / 1e12, "query_mse": qmse,
        "config": {"workload": f"BASELINE config 5 share: {tasks} of 64 tasks x B={cfg.batch} x T={d.window_size} x "
                               f"N={d.num_nodes} x C={d.input_channels}, Hc={d.hidden_channels}, LSTM "
                               f"{d.lstm_num_layers}x{d.lstm_hidden_size}, K={cfg.inner_steps} inner steps",
                   "tasks": tasks, "so_kept_steps": kept, "task_groups": groups},
        "rank_workload": rank_workload(d, cfg, tasks, 5),
    }
    if kern is not None:
        out.update(kernel_report(kern, steps, elapsed, out["rank_workload"]))
    return out


TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic.json")

# timing category -> the kernel symbol its HIP-event brackets enclose
KERNEL_SYMBOL = {"gcn_layer": "k_gcn_layer|k_gcn_mlp", "lstm_fwd_step": "k_lstm_fwd_step", "lstm_fwd_dual": "k_lstm_fwd_dual",
                 "head_loss": "k_head_loss|k_head_dual", "head_dh": "k_gemm_nn|k_gemm_nn_dual",
                 "lstm_bwd_step": "k_lstm_bwd_step", "lstm_bwd_dual": "k_lstm_bwd_dual", "wgrad": "k_wgrad",
                 "wgrad_reduce": "k_wgrad_reduce", "xg_proj": "k_xg_dedup|k_gemm_nt",
                 "dg_rowsum": "k_dg_rowsum"}


def rank_workload(d, cfg, rank_tasks, config=2):
    """Key of a per-rank workload in profiles/traffic.json: what one rank runs per meta-step (its
    task count sets the task groups and so the per-launch bytes; at N=1 it is the whole meta-batch,
    at N>1 rank 0's round-robin share, the largest)."""
    return (f"BASELINE config {config} rank workload: {rank_tasks} tasks x B={cfg.batch} x T={d.window_size} x "
            f"N={d.num_nodes} x C={d.input_channels}, Hc={d.hidden_channels}, LSTM {d.lstm_num_layers}x"
            f"{d.lstm_hidden_size}, K={cfg.inner_steps} inner steps, order {cfg.order}")


def measured_traffic(category, rank_key):
    """Per-launch HBM bytes of a timing category from the committed PMC profiles
    (tools/prof_summary.py output), only when one was taken on this exact per-rank workload
    (rank_workload). PMC counters cannot be read from inside a timed run, so the figure comes from
    separate rocprofv3 --pmc passes of a one-GPU bench run with the same per-rank task count."""
    if not os.path.exists(TRAFFIC_JSON):
        return None
    try:
        t = json.load(open(TRAFFIC_JSON))
    except (OSError, ValueError):
        return None
    prof = t.get("profiles", {}).get(rank_key)
    if not prof or category not in prof.get("categories", {}):
        return None
    c = dict(prof["categories"][category])
    c["source"] = prof.get("profile") or "profiles/traffic.json"
    return c


def kernel_report(kern, steps, elapsed, rank_key):
    """Per-category kernel times of the timed region (HIP events on the launch stream), the executed
    flops (each launch's count is what its kernel actually computes -- GCN rows of consecutive windows
    once per distinct stream row, no recurrent products at t = 0, tangent-only passes of kept steps --
    beside SURVEY §8(d)'s convention, which counts the GCN once per sample-step), and the roofline of
    the dominant kernel: its average launch's flops over its average launch duration, with the HBM
    bytes per launch from the committed PMC passes of the same per-rank workload."""
    from weatherforecast_stgcn_maml_amd import _capi

    forms = _capi.product_forms()
    executed = sum(v["flops"] for k, v in kern.items() if not k.endswith("_wall")) / steps
    out = {"executed_tflop": executed / 1e12,
           "achieved_tflops_executed": executed / (elapsed / steps) / 1e12,
           "executed_flops_basis": "sum of the flops of every timed launch (what each kernel computes; the "
                                   "deduplicated GCN rows once, no h_{-1} = 0 products, tangent-only kept steps)"}
    # each timing category is one kernel symbol (api.cpp enum Cat); the roofline is quoted for the one
    # with the most time: its average launch duration here must match rocprofv3's for that symbol
    dom = max((k for k in kern if k not in ("misc", "wgrad_reduce", "xg_proj", "dg_rowsum") and not k.endswith("_wall")
               and not (kern.get(k + "_wall", {}).get("launches"))), key=lambda k: kern[k]["ms"])
    kd = kern[dom]
    ach = kd["flops"] / (kd["ms"] * 1e-3) / 1e12 if kd["ms"] > 0 else 0.0
    traffic = measured_traffic(dom, rank_key)
    x6 = forms.get(CAT_FAMILY.get(dom, ""), 0) > 0
    peak = PEAK_X6_TFLOPS if x6 else PEAK_FP32_MFMA_TFLOPS
    roof = {
        "kernel": KERNEL_SYMBOL.get(dom, dom), "category": dom, "bound": "mfma", "achieved": ach, "peak": peak,
        "unit": "TFLOP/s", "frac": ach / peak,
        "peak_basis": ("f32 work as six bf16 piece products: dense BF16 MFMA 2516.8 TF / 6 (the native f32 MFMA "
                       "peak is 157.3 TF)" if x6 else "v_mfma_f32_32x32x2_f32 dense peak"),
        "traffic": traffic["bytes_per_launch"] if traffic else None,
        "avg_launch_us": kd["ms"] * 1e3 / max(kd["launches"], 1),
        "flops_per_launch": kd["flops"] / max(kd["launches"], 1),
    }
    if traffic:
        roof["traffic_unit"] = "bytes/launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE)"
        roof["traffic_source"] = traffic["source"]
        roof["hbm_tbs"] = traffic["bytes_per_launch"] / (roof["avg_launch_us"] * 1e-6) / 1e12
    out["roofline"] = roof
    out["kernels"] = {k: {"ms_per_step": v["ms"] / steps,
                          "tflops": (v["flops"] / (v["ms"] * 1e-3) / 1e12) if v["ms"] > 0 else 0.0,
                          "launches_per_step": v["launches"] / steps}
                      for k, v in kern.items() if v["launches"] > 0}
    # every major category against both roofs: its f32-work rate over the product form's MFMA peak and its
    # HBM bytes (committed PMC passes of this workload, per launch x launches) over 8 TB/s; categories whose
    # sweeps ran as concurrent row chunks are timed by their sweeps' wall (<cat>_wall), not the summed chunks
    rl = {}
    for k, v in kern.items():
        if k.endswith("_wall") or k == "misc" or v["launches"] == 0:
            continue
        wall = kern.get(k + "_wall", {})
        t_ms = wall["ms"] if wall.get("launches") else v["ms"]
        if t_ms <= 0:
            continue
        fam = CAT_FAMILY.get(k)
        pk = (PEAK_X6_TFLOPS if forms.get(fam, 0) > 0 else PEAK_FP32_MFMA_TFLOPS) if fam else None
        tf = v["flops"] / (t_ms * 1e-3) / 1e12
        e = {"ms_per_step": t_ms / steps, "timed_by": "sweep wall" if wall.get("launches") else "kernel events",
             "tflops": tf, "mfma_frac": (tf / pk) if (pk and v["flops"] > 0) else None}
        tr = measured_traffic(k, rank_key)
        if tr:
            gbs = tr["bytes_per_launch"] * v["launches"] / (t_ms * 1e-3) / 1e9
            e.update({"hbm_bytes_per_launch": tr["bytes_per_launch"], "hbm_tbs": gbs / 1e3, "hbm_frac": gbs / PEAK_HBM_GBS})
        rl[k] = e
    out["rooflines"] = rl
    out["whole_step_executed_frac"] = out["achieved_tflops_executed"] / PEAK_X6_TFLOPS
    out["rooflines_note"] = ("per category: mfma_frac = f32-work TFLOP/s / the product form's MFMA peak (419.5 for "
                             "bf16x6); hbm_frac = PMC bytes per launch (profiles/traffic.json, this workload) x "
                             "launches / time / 8 TB/s; whole_step_executed_frac = executed TFLOP/s / 419.5")
    if any(k.endswith("_wall") for k in out["kernels"]):
        out["kernels_note"] = ("LSTM sweeps whose diagonals ran as concurrent row chunks on side streams (options "
                               "bptt_streams / fwd_streams): their category's ms sums the chunks' kernel times, which "
                               "overlap; <category>_wall is the sweeps' wall time (its launches count sweeps)")
    return out


def relaunch(args) -> int:
    """``--gpus N`` without a torch.distributed launcher: start N ranks (one per GPU) through
    torch.distributed.run as a child process, before this process touches the GPU, and return
    its exit code (never an exec: see the contract in the module docstring)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ.get('WORLD_SIZE')} but --gpus {args.gpus}")
    import torch
    import torch.distributed as dist

    from weatherforecast_stgcn_maml_amd import synth
    from weatherforecast_stgcn_maml_amd.config import SEED, MamlConfig, ModelDims
    from weatherforecast_stgcn_maml_amd.graph import build_spatial_graph
    from weatherforecast_stgcn_maml_amd.maml import MetaLearner, shard_tasks, stream_len_for

    from weatherforecast_stgcn_maml_amd.distributed import env_rank, init_from_env, max_over_ranks, min_over_ranks

    from weatherforecast_stgcn_maml_amd import _capi

    rank, world, local = env_rank()
    # one process per GPU; SMAML_DIST_BACKEND=gloo + LOCAL_RANK mod device count lets a
    # single-GPU box rehearse the N>1 path (the driver's 8-GPU runs use RCCL, one GPU each)
    dev_idx = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_idx)
    backend = os.environ.get("SMAML_DIST_BACKEND", "nccl")
    init_from_env(backend, torch.device("cuda", dev_idx))
    local = dev_idx

    d = ModelDims(num_nodes=args.nodes, hidden_channels=args.hidden_channels or 256)
    cfg = MamlConfig(inner_steps=args.inner_steps, batch=args.batch, order=args.order)
    side = int(round(d.num_nodes ** 0.5))
    lats, lons = synth.region_grid(n_lat=side, n_lon=side)
    ei, _, _ = build_spatial_graph(lats, lons, 4)
    P = synth.init_params(SEED, d)
    names = [k for k in P if k.startswith(("lstm.", "output_layer."))]
    mine = shard_tasks(args.tasks, rank, world)
    T_total = stream_len_for(cfg, d)
    feats = [synth.make_features(synth.task_seed(j), d.num_nodes, T_total) for j in mine]
    # ranks sharing one GPU (the N>1 rehearsal on a one-GPU box) each plan task groups for their share of HBM
    per_dev = -(-world // max(1, torch.cuda.device_count()))
    ml = MetaLearner(d, cfg, {k: v for k, v in P.items() if k not in names}, {k: P[k] for k in names},
                     ei, device=f"cuda:{local}", task_group=args.task_group, dropout=tuple(args.dropout),
                     dropout_seed=SEED, mem_share=1.0 / per_dev)
    ml.set_tasks(feats, task_ids=mine)
    torch.cuda.synchronize()

    progress(f"rank {rank}: {len(mine)} tasks, warmup")
    for _ in range(args.warmup):
        ml.meta_step(sync=False)
    if not args.no_timing:
        ml.ctx.timing_collect()  # drop warmup records
        ml.ctx.timing(True)
    ml.comm_timing = world > 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    res = None
    for _ in range(args.steps):
        res = ml.meta_step(sync=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    progress(f"rank {rank}: timed region done")
    ml.ctx.sync(_capi.stream_ptr(torch))  # a timed-out grid-barrier kernel would have invalidated the run: raise
    kern = None
    if not args.no_timing:
        ml.ctx.timing(False)
        kern = ml.ctx.timing_collect()
    qsum = float(res.losses[-1].sum().item()) if len(mine) else 0.0
    qmse = qsum / max(len(mine), 1)
    comm = None
    hung = False  # the N>1 C-ABI RCCL check outlived its watchdog
    if world > 1:
        ar_ms, ar_n = ml.comm_time_collect()
        ml.comm_timing = False
        comm = {
            "allreduce_ms": max_over_ranks(ar_ms / max(ar_n, 1), f"cuda:{local}"),
            "allreduce_ms_min_rank": min_over_ranks(ar_ms / max(ar_n, 1), f"cuda:{local}"),
            "elapsed_min_ms": min_over_ranks(elapsed, f"cuda:{local}") * 1e3,
            "elapsed_max_ms": max_over_ranks(elapsed, f"cuda:{local}") * 1e3,
        }
        elapsed = max_over_ranks(elapsed, f"cuda:{local}")
        q = torch.tensor([qsum], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(q)
        qmse = float(q.item()) / args.tasks
        capi_comm = os.environ.get("SMAML_BENCH_CAPI_COMM", "1")  # 0 = skip, force = also under gloo
        if (backend == "nccl" and capi_comm != "0") or capi_comm == "force":
            # after the timed region: the C ABI's own RCCL communicator (smaml_comm_*) across
            # the same ranks, on a buffer the size of the meta-step's one all-reduce
            # Its init is bounded by comm_timeout_ms, its collectives are not: run it on a daemon
            # thread and, past CAPI_COMM_WATCHDOG_S, report the timeout in the line and leave
            # without the (possibly blocked) teardown, so a hung check never costs the headline.
            import threading

            from weatherforecast_stgcn_maml_amd.distributed import capi_comm_check
            box = {}

            def check():
                torch.cuda.set_device(local)
                try:
                    box["r"] = capi_comm_check(ml.ctx, ml.theta.numel() + 64)
                except Exception as e:  # noqa: BLE001 - reported in the line; the headline is already measured
                    box["r"] = {"status": f"error: {e}", "world": world}

            th = threading.Thread(target=check, daemon=True)
            th.start()
            th.join(CAPI_COMM_WATCHDOG_S)
            comm["capi_comm_check"] = box.get("r") or {
                "status": f"error: no result within {CAPI_COMM_WATCHDOG_S} s (left without teardown)", "world": world}
            hung = th.is_alive()

    ms_per_step = elapsed / args.steps * 1e3
    value = args.steps / elapsed
    flops_meta = algorithmic_flops(d, args.tasks, cfg.inner_steps, cfg.batch, cfg.order)
    out = {
        "metric": "MAML meta-steps/sec (15-task batch, N=441, T=24)" if args.config == 2 else
                  "MAML meta-steps/sec (BASELINE config 5 stress: 64 tasks, N=1024, Hc=512, K=10)",
        "value": value,
        "unit": "meta-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",  # f32 operands and accumulation; products f32 MFMA or f32-accurate bf16x6 (config.products)
        "data": "synthetic ERA5-shaped feature streams (numpy PCG64 seeds 1000+j), random-init weights",
        "config": {
            "workload": f"BASELINE config {args.config}: {args.tasks} tasks x B={cfg.batch} x T={d.window_size} x "
                        f"N={d.num_nodes} x C={d.input_channels}, Hc={d.hidden_channels}, "
                        f"LSTM {d.lstm_num_layers}x{d.lstm_hidden_size}, K={cfg.inner_steps} inner steps",
            "tasks": args.tasks, "batch": cfg.batch, "inner_steps": cfg.inner_steps,
            "maml_order": cfg.order,
            "parallelism": (f"task-sharded x{world} + one {'RCCL' if backend == 'nccl' else backend} all-reduce "
                            f"per meta-step" if world > 1 else "single GPU, no collective"),
            "gcn_hoist": "GCN features computed once per distinct sample per meta-step (F2); the rows t >= 1 "
                         "of a batch of consecutive windows once per distinct stream row (F3, option gcn_dedup, "
                         "bitwise equal); meta_step_tflop counts the GCN once per sample-step (SURVEY 8d), "
                         "executed_tflop counts what ran",
            "so_kept_steps": ml.ctx.so_kept_steps() if cfg.order == 2 else 0,
            "task_group": len(ml._groups[0][1]) if ml._groups else 0,
            "dropout": list(args.dropout),
            "products": _capi.build_info(),
        },
        "rank_workload": rank_workload(d, cfg, len(mine), args.config),
        "meta_step_tflop": flops_meta / 1e12,
        "achieved_tflops_whole_step": flops_meta / (elapsed / args.steps) / 1e12,
        "query_mse": qmse,
    }
    if kern is not None:
        out.update(kernel_report(kern, args.steps, elapsed, out["rank_workload"]))
    if comm is not None:
        # the all-reduce's exposed time per meta-step (HIP events on the compute stream: end of this
        # rank's meta-step work -> reduced buffer ready, incl. waiting for the slowest rank), max /
        # min over ranks, and every rank's own elapsed time over the timed region
        out["collective"] = dict(comm, what="one all_reduce(SUM) of [meta-gradient | query-loss sum], "
                                            f"{(ml.theta.numel() + 64) * 4 / 1e6:.2f} MB, per meta-step")
    if rank == 0 and world == 1 and args.cpu_sample_steps > 0:
        t_step, cores, n_os, n_aff = cpu_baseline(d, args.cpu_sample_steps, P, ei, feats[0])
        sample_steps = args.tasks * (cfg.inner_steps + 1) * cfg.batch
        out["cpu_baseline"] = {
            "value": 1.0 / (sample_steps * t_step), "unit": "meta-steps/s", "cores": cores,
            "os_cpu_count": n_os, "affinity_cpus": n_aff, "kind": "port",
            "sample": f"{args.cpu_sample_steps} batch-1 sample-steps (fwd+bwd+clip+SGD) of the reference's "
                      f"per-node nn.LSTM CPU path at N={d.num_nodes}, {t_step:.3f} s each; meta-steps/s = "
                      f"1/({sample_steps} sample-steps x t); first-order work only (the reference has no "
                      f"second-order path); the port times 1.04x the reference's own inner step on the "
                      f"same sample (profiles/r02_cpu_calibration.log)",
        }
        out["vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
    if world == 1 and args.adapt_epochs > 0 and args.config == 2:
        # BASELINE config 4, after (never inside) the headline timed region, on a fresh context
        ml.ctx.close()
        del ml
        torch.cuda.empty_cache()
        progress("config 4 adaptation")
        ad, _ = adaptation_bench(ModelDims(num_nodes=441, hidden_channels=256), P, ei, epochs=args.adapt_epochs)
        out["adaptation"] = ad
    if world == 1 and args.cfg5_share_tasks > 0 and args.config == 2:
        if "ml" in locals():
            ml.ctx.close()
            del ml
            torch.cuda.empty_cache()
        progress("config 5 rank share")
        out["config5_rank_share"] = config5_share_bench(args.cfg5_share_tasks, timing=not args.no_timing)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if hung:
        # the check's thread is still inside a collective: a teardown could block on it
        sys.stderr.flush()
        os._exit(0)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
