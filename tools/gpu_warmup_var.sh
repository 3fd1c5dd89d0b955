#!/usr/bin/env bash
# K=20 step time against the warm-up length (timed-region stall study), no profiler.
set -u
mkdir -p gpurun_out/wv
for w in 5 5 2 10 10 20 40; do
  timeout -k 10 200 python3 bench.py --warmup $w --steps 20 --cpu-baseline 0 --fwd-only 0 > gpurun_out/wv/o.log 2>&1 || { tail -3 gpurun_out/wv/o.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/wv/o.log').read().strip().splitlines()[-1]); print('W=$w', d['ms_per_step'], d['host_launch_ms'])" | tee -a gpurun_out/wv/summary.txt
done
