#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6g
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6g/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6g/kt_det.log 2>&1 || { tail -5 gpurun_out/r6g/kt_det.log; exit 1; }
f=$(find gpurun_out/r6g/kt_det -name "*kernel_stats.csv" | head -1); echo $f
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(f"{r['Name'][:60]:60s} n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.2f}us tot={float(r['TotalDurationNs'])/1e6:8.3f}ms")
PY
timeout -k 10 300 python3 bench.py --deterministic 1 --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6g/bench_det_k20.log 2>&1 || { tail -5 gpurun_out/r6g/bench_det_k20.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6g/bench_det_k20.log').read().strip().splitlines()[-1]);print('det K20 ms/step', d['ms_per_step'])"
