#!/bin/bash
# data-parallel rehearsal on one GPU as rank 0 of W = 8 (bench.py --rehearse-world): compute only
# (infinite links), device copies of the exchange bytes, and modelled links (350 / 537 GB/s + 10 us
# per collective)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rh
for args in "--rehearse-comm model --link-gbps 1e9 --link-latency-us 0" "--rehearse-comm copy" "--rehearse-comm model" "--rehearse-comm model --link-gbps 537"; do
  timeout -k 10 300 python3 bench.py --rehearse-world 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 $args > gpurun_out/rh/out.json 2> gpurun_out/rh/err.log || { echo "failed: $args"; tail -10 gpurun_out/rh/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rh/out.json')); print('$args ->', d['ms_per_step'], d.get('kernels_ms',{}).get('adam'), d.get('rehearsal'))" | cut -c1-300
done
