#!/bin/bash
# round 6: bench's peer-exchange legs (N=2 over gloo on one GPU, the W=8 rehearsal) and the rehearsal numbers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6p2
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_dp.py -x -v --timeout 500 --timeout-method thread -rA > gpurun_out/r6p2/bench_dp.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/r6p2/bench_dp.log | head -30
[ $rc = 0 ] || exit $rc
B="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --fwd32-line 0 --parity 0 --steps 200 --warmup 20 --rehearse-world 8"
timeout -k 10 300 $B --rehearse-comm peer > gpurun_out/r6p2/reh_peer.json 2> gpurun_out/r6p2/reh_peer.err || exit 1
timeout -k 10 300 $B --rehearse-comm model --link-gbps 537 --link-latency-us 10 > gpurun_out/r6p2/reh_537.json 2> gpurun_out/r6p2/reh_537.err || exit 1
timeout -k 10 300 $B --rehearse-comm copy > gpurun_out/r6p2/reh_copy.json 2> gpurun_out/r6p2/reh_copy.err || exit 1
for f in reh_peer reh_537 reh_copy; do python3 -c "
import json,sys; d=json.load(open('gpurun_out/r6p2/$f.json')); print('$f', d['ms_per_step'], d.get('dp_kernels_ms'), d.get('peer_status'))"; done
