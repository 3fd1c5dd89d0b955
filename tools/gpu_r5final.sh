#!/bin/bash
# round-5 final set at HEAD: the GPU suite, smoke, the measurement set (tools/gpu_round_measure.sh),
# the driver-shaped K=20 line and the multi-view line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fin5
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/fin5/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " gpurun_out/fin5/tests.log | head -30; exit 1; }
tail -1 gpurun_out/fin5/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin5/smoke.log 2>&1 || { tail -5 gpurun_out/fin5/smoke.log; exit 1; }
tail -1 gpurun_out/fin5/smoke.log
bash tools/gpu_round_measure.sh || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/m/bench_k20.log 2>&1 || { tail -5 gpurun_out/m/bench_k20.log; exit 1; }
timeout -k 10 300 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/m/bench_mv.log 2>&1 || { tail -5 gpurun_out/m/bench_mv.log; exit 1; }
for f in bench_bf16 bench_fp32 bench_uniform bench_k20 bench_mv; do python3 -c "import json;d=json.loads(open('gpurun_out/m/$f.log').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],d['value'])"; done
