#!/bin/bash
# round 5 measurement set at HEAD (tools/gpu_round_measure.sh) + the driver-shaped K=20 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round_measure.sh || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/m/bench_k20.log 2>&1 || { tail -5 gpurun_out/m/bench_k20.log; exit 1; }
tail -1 gpurun_out/m/bench_k20.log | cut -c1-200
