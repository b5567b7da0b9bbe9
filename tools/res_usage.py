"""Per-kernel VGPR / AGPR / scratch / occupancy of the library sources (gfx950), H=128 instances.
Usage: python tools/res_usage.py [-DSMAML_X=1 ...]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(REPO, "weatherforecast_stgcn_maml_amd", "csrc")
for f in ("kernels", "kernels_dual"):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(REPO, "include"),
                        "-I", CS, *sys.argv[1:], "-c", os.path.join(CS, f + ".hip"), "-o", f"/tmp/res_{f}.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur = None
    rows = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for c in rows:
        n = c["name"]
        if re.search(r"^_ZN5smaml\d+k_[a-z_]+ILi(32|64|256)E", n):
            continue
        short = re.sub(r"^_ZN5smaml\d+", "", n)[:int(os.environ.get("RES_W", "48"))]
        print(f"{short:48s} vgpr {c.get('VGPRs', '?'):>4s} agpr {c.get('AGPRs', '?'):>4s} "
              f"scratch {c.get('ScratchSize [bytes/lane]', '?'):>3s} occ {c.get('Occupancy [waves/SIMD]', '?'):>2s} "
              f"lds {c.get('LDS Size [bytes/block]', '?')}")
