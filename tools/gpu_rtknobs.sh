#!/usr/bin/env bash
# HIP runtime submission knobs vs the timed region's tail stall (K-step graph, node ~215 onwards).
set -u
mkdir -p gpurun_out/rt
for e in "X=0" "ROC_AQL_QUEUE_SIZE=65536" "DEBUG_HIP_GRAPH_BATCH_SIZE=4096" "DEBUG_CLR_MAX_BATCH_SIZE=4096" "DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  for k in 20 200; do
    env $e timeout -k 10 200 python3 bench.py --warmup 10 --steps $k --cpu-baseline 0 --fwd-only 0 > gpurun_out/rt/o.log 2>&1 || { echo "$e $k FAILED"; tail -3 gpurun_out/rt/o.log; continue; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/rt/o.log').read().strip().splitlines()[-1]); print('$e', $k, d['ms_per_step'], d['host_launch_ms'], d['final_loss'])" | tee -a gpurun_out/rt/summary.txt
  done
done
