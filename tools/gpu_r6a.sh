#!/bin/bash
# round 6, first call: where two eager default-schedule DP runs part ways (tools/dp_divergence.py),
# and the bench line's new parity_vs_oracle leg on a short run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6a
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 128 1 > gpurun_out/r6a/div.log 2>&1 || { tail -20 gpurun_out/r6a/div.log; exit 1; }
head -3 gpurun_out/r6a/div.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-seconds 2 > gpurun_out/r6a/bench.log 2>&1 || { tail -5 gpurun_out/r6a/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6a/bench.log').read().strip().splitlines()[-1]);print(d['ms_per_step']);print(json.dumps(d['cpu_baseline'].get('parity_vs_oracle'),indent=1))"
