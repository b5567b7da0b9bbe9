#!/bin/bash
# Does rocprofv3 crash at exit for ANY torch process here, or only for the bench? (diagnostic)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/probe_kt -o run -- python -c "import torch; x = torch.ones(1 << 20, device='cuda'); print(float((x * 2).sum()))" > gpurun_out/probe.log 2>&1
echo "trivial torch under rocprofv3: rc $?"
