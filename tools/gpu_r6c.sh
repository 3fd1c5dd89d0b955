#!/bin/bash
# round 6: the deterministic sort rewrite (tests + timing), then the DP divergence diagnostics
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops_bwd.py -k csc_transpose tests/test_gpu_deterministic.py tests/test_gpu_graph.py > gpurun_out/r6c/tests.log 2>&1 || { tail -30 gpurun_out/r6c/tests.log; exit 1; }
tail -2 gpurun_out/r6c/tests.log
timeout -k 10 300 python3 bench.py --deterministic 1 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6c/bench_det.log 2>&1 || { tail -5 gpurun_out/r6c/bench_det.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6c/bench_det.log').read().strip().splitlines()[-1]);print('det ms/step', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_det -o det -- python3 bench.py --deterministic 1 --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6c/prof_det.log 2>&1 || { tail -5 gpurun_out/r6c/prof_det.log; exit 1; }
find /tmp/prof_det -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6c/det_kernel_stats.csv \;
head -14 gpurun_out/r6c/det_kernel_stats.csv | cut -c1-160
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 128 1 0 > gpurun_out/r6c/div_fresh.log 2>&1 || { tail -20 gpurun_out/r6c/div_fresh.log; exit 1; }
grep "^#" gpurun_out/r6c/div_fresh.log
timeout -k 10 300 python3 -u tools/dp_divergence.py 4 128 1 1 > gpurun_out/r6c/div_warm.log 2>&1 || { tail -20 gpurun_out/r6c/div_warm.log; exit 1; }
grep "^#" gpurun_out/r6c/div_warm.log
