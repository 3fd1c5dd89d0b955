#!/bin/bash
# round 6 (resumed session): GPU suite + smoke + the driver-shaped bench at HEAD on a fresh build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6r
bash tools/gpu_r6_suite.sh > gpurun_out/r6r/suite.txt 2>&1; rc=$?
cat gpurun_out/r6r/suite.txt
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6r/bench_k20.json 2> gpurun_out/r6r/bench_k20.err || exit 1
cut -c1-400 gpurun_out/r6r/bench_k20.json
