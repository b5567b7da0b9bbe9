"""Grid sizing of the grid-barrier bookkeeping kernels (kernels.h grid_barrier_grid):
a quarter of the resident capacity at most, never more blocks than items, 0 when the capacity is
unknown (two-launch fallback), and the debug oversize grid strictly above the capacity. Compiled
host-only from the library's own header and run on the CPU."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "weatherforecast_stgcn_maml_amd", "csrc")


def _hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    return None


@pytest.mark.skipif(_hipcc() is None, reason="needs hipcc")
def test_grid_barrier_sizing(tmp_path):
    exe = tmp_path / "gb_check"
    subprocess.run([_hipcc(), "--offload-arch=gfx950", "--cuda-host-only", "-O1", "-std=c++17", "-I", CSRC,
                    "-I", os.path.join(REPO, "include"), os.path.join(REPO, "tools", "grid_barrier_plan_check.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all passed" in r.stdout
