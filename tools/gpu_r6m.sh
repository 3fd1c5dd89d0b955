#!/bin/bash
# round 6: plan option FWD32 (fp32-accurate forward, bf16 backward): tests, bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6m
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fwd32.py > gpurun_out/r6m/tests.log 2>&1 || { grep -E "FAIL|Error|assert|relative L2" gpurun_out/r6m/tests.log | head -20; tail -3 gpurun_out/r6m/tests.log; exit 1; }
grep -E "PASS|relative L2|passed" gpurun_out/r6m/tests.log
for k in 20 200; do w=$([ $k = 20 ] && echo 5 || echo 20)
timeout -k 10 300 python3 bench.py --fwd32 1 --steps $k --warmup $w --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd32-line 0 > gpurun_out/r6m/bench_k$k.log 2>&1 || { tail -5 gpurun_out/r6m/bench_k$k.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6m/bench_k$k.log').read().strip().splitlines()[-1]);print('fwd32 K$k', d['ms_per_step'], d['schedule'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6m/kt -o run -- python3 bench.py --fwd32 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd32-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6m/kt.log 2>&1 || { tail -5 gpurun_out/r6m/kt.log; exit 1; }
