#!/usr/bin/env bash
# Round-end measurement refresh: kernel stats of the headline run, the default bench line (with the
# CPU baseline) and the driver-shaped K=20 / W=5 line.  Every GPU step under its own limit.
set -eu
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/kt -o run \
  -- python3 bench.py --steps 48 --warmup 8 --cpu-baseline 0 --fwd-only 0 > gpurun_out/fin/kt.log 2>&1
echo "kt ok"
timeout -k 10 400 python3 bench.py > gpurun_out/fin/bench_bf16.log 2>&1
echo "bench ok"
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/fin/bench_bf16_k20.log 2>&1
echo "k20 ok"
