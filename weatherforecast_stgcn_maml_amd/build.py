"""Build libsmaml.so in-tree with hipcc for gfx950 (cross-compiles without a GPU)."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = [os.path.join(CSRC, "kernels.hip"), os.path.join(CSRC, "kernels_dual.hip"),
           os.path.join(CSRC, "kernels_gcn.hip"), os.path.join(CSRC, "kernels_small.hip"),
           os.path.join(CSRC, "api.cpp")]
HEADERS = [os.path.join(CSRC, "gemm_core.h"), os.path.join(CSRC, "kernels.h"), os.path.join(CSRC, "loaders.h"),
           os.path.join(REPO, "include", "smaml.h")]
OUT = os.path.join(HERE, "libsmaml.so")
ARCH = os.environ.get("SMAML_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


STAMP = OUT + ".flags"  # the extra flags the default library was built with (build-flag changes rebuild it)


def extra_flags() -> list:
    return os.environ.get("SMAML_EXTRA_FLAGS", "").split()


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    try:
        with open(STAMP) as f:
            if f.read() != " ".join(extra_flags()):
                return False
    except OSError:
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    """Compile libsmaml.so (one hipcc per translation unit, in parallel, then link);
    ``defines`` (e.g. ["SMAML_GATE_BK=16"]) build A/B variants."""
    if not force and not defines and out == OUT and up_to_date():
        return out
    # -fno-slp-vectorize: keeps the bf16x6 split's f32 subtractions as v_sub_f32 instead of v_pk_add_f32
    # (packed f32 VALU beside MFMAs costs extra issue cycles; A/B 2045 -> 2003 ms per meta-step)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", "-I", os.path.join(REPO, "include"),
             "-I", CSRC, *[f"-D{d}" for d in defines], *extra_flags()]
    objs, procs = [], []
    try:
        for src in SOURCES:
            obj = f"{out}.{os.path.basename(src)}.o"
            cmd = [hipcc(), *flags, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            procs.append(subprocess.Popen(cmd))
            objs.append(obj)
        rcs = [p.wait() for p in procs]
        if any(rcs):
            raise subprocess.CalledProcessError(max(rcs), "hipcc")
        link = [hipcc(), f"--offload-arch={ARCH}", "-shared", *objs, "-o", out + ".tmp"]
        if verbose:
            print(" ".join(link))
        subprocess.run(link, check=True)
        os.replace(out + ".tmp", out)
        if out == OUT:
            with open(STAMP, "w") as f:
                f.write(" ".join(extra_flags()))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for o in objs + [out + ".tmp"]:
            if os.path.exists(o):
                os.remove(o)
    return out


if __name__ == "__main__":
    print(build(force=True, verbose=True))
