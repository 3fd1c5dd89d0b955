#!/bin/bash
# round 6: the divergence diagnostics, fresh and warm Adam state
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6b
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 128 1 0 > gpurun_out/r6b/div_fresh.log 2>&1 || { tail -20 gpurun_out/r6b/div_fresh.log; exit 1; }
grep "^#" gpurun_out/r6b/div_fresh.log
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 128 1 1 > gpurun_out/r6b/div_warm.log 2>&1 || { tail -20 gpurun_out/r6b/div_warm.log; exit 1; }
grep "^#" gpurun_out/r6b/div_warm.log
