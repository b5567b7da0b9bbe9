"""Interleaved A/B of bench.py variants on one GPU box. Each variant = (name, library, extra env);
every round runs every variant once in its own process (bench.py --steps S --warmup 1, no CPU
baseline, no adaptation / config-5 extras), then a per-kernel table of the best run of each variant.

usage: ab_run.py OUT_LOG ROUNDS NAME=LIB[:K=V[;K=V...]] ...   (LIB relative to the package dir)
"""
import json
import os
import subprocess
import sys

out, rounds, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "weatherforecast_stgcn_maml_amd")
variants = []
for sp in specs:
    name, _, rest = sp.partition("=")
    lib, _, envs = rest.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(";") if kv)
    variants.append((name, os.path.join(pkg, lib), env))
steps = os.environ.get("AB_STEPS", "2")
extra = os.environ.get("AB_BENCH_ARGS", "").split()
res = {n: [] for n, _, _ in variants}
with open(out, "w") as log:
    for r in range(rounds):
        for name, lib, env in variants:
            e = dict(os.environ, SMAML_LIB=lib, **env)
            cmd = [sys.executable, "bench.py", "--steps", steps, "--warmup", "1", "--cpu-sample-steps", "0",
                   "--adapt-epochs", "0", "--cfg5-share-tasks", "0", *extra]
            p = subprocess.run(["timeout", "-k", "10", "300", *cmd], env=e, capture_output=True, text=True)
            if p.returncode != 0:
                log.write(f"{name} FAILED rc={p.returncode}\n{p.stdout[-3000:]}\n{p.stderr[-3000:]}\n")
                log.flush()
                print(f"{name} FAILED rc={p.returncode}", flush=True)
                sys.exit(p.returncode)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
            log.write(f"{name} {line}\n")
            log.flush()
            j = json.loads(line)
            res[name].append(j)
            print(f"round {r} {name}: {j['ms_per_step']:.1f} ms", flush=True)
cats = None
for name, rs in res.items():
    cats = cats or [c for c in rs[0].get("kernels", {})]
    ms = sorted(x["ms_per_step"] for x in rs)
    ks = {c: min(x["kernels"][c]["ms_per_step"] for x in rs) for c in cats}
    print(f"{name:14s} step {ms[0]:8.1f} ms (max {ms[-1]:8.1f}) | " +
          " ".join(f"{c} {ks[c]:.0f}" for c in cats if ks[c] > 1), flush=True)
