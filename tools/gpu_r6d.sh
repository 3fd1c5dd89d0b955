#!/bin/bash
# round 6: the rewritten default-schedule DP graph test; deterministic-mode kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6d
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wire.py -k "default_schedule" > gpurun_out/r6d/tests.log 2>&1 || { tail -30 gpurun_out/r6d/tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6d/tests.log | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6d/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6d/kt_det.log 2>&1 || { tail -5 gpurun_out/r6d/kt_det.log; exit 1; }
find gpurun_out/r6d/kt_det -name "*kernel_stats.csv" | head -2
timeout -k 10 300 python3 bench.py --deterministic 1 --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6d/bench_det_k20.log 2>&1 || { tail -5 gpurun_out/r6d/bench_det_k20.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6d/bench_det_k20.log').read().strip().splitlines()[-1]);print('det K20 ms/step', d['ms_per_step'])"
