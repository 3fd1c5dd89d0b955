#!/bin/bash
# round 6: rocprofv3 kernel-trace stats of the W=8 peer-store rehearsal (rank 0's kernels, K=48)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp/kt -o run -- python3 bench.py --rehearse-world 8 --rehearse-comm peer --steps 48 --warmup 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --fwd32-line 0 --parity 0 > gpurun_out/pp/kt.log 2>&1 || { tail -5 gpurun_out/pp/kt.log; exit 1; }
python3 -c "
import csv
for x in csv.DictReader(open('gpurun_out/pp/kt/run_kernel_stats.csv')): print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,2))" | head -20
