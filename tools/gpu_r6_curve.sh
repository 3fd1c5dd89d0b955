#!/bin/bash
# round 6: the one-GPU rehearsal of rank 0 at W = 2 / 4 / 8 for the RCCL schedule (links modelled at 537 GB/s
# + 10 us per collective, tail in the all-to-all's group) and the peer-store exchange (no link time)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/curve
R="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --fwd32-line 0 --parity 0"
for w in 2 4 8; do
  timeout -k 10 300 $R --rehearse-world $w --link-gbps 537 --plan-option TAIL_IN_A2A=1 > gpurun_out/curve/rccl537_w$w.log 2>&1 || { tail -3 gpurun_out/curve/rccl537_w$w.log; exit 1; }
  timeout -k 10 300 $R --rehearse-world $w --rehearse-comm peer > gpurun_out/curve/peer_w$w.log 2>&1 || { tail -3 gpurun_out/curve/peer_w$w.log; exit 1; }
  for f in rccl537_w$w peer_w$w; do python3 -c "import json;d=json.loads(open('gpurun_out/curve/$f.log').read().strip().splitlines()[-1]);k=d.get('dp_kernels_ms',{});print('$f',d['ms_per_step'],{x:k.get(x) for x in ('grad_pass','all_to_all','adam','all_gather','shadow_rebuild')})"; done
done
