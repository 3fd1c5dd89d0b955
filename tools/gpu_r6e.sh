#!/bin/bash
# round 6: divergence of the default DP schedule from warm Adam states of several v
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6e
for v in 1e-6 1e-4; do
for bc in "128 1" "96 3"; do
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 $bc $v > gpurun_out/r6e/div_${v}_${bc// /_}.log 2>&1 || { tail -20 gpurun_out/r6e/div_${v}_${bc// /_}.log; exit 1; }
grep "^# [tfgu]" gpurun_out/r6e/div_${v}_${bc// /_}.log
done
done
