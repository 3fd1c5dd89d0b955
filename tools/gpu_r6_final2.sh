#!/bin/bash
# round 6 closing set, part A (part B: tools/gpu_round_measure.sh): GPU suite + smoke, the driver-shaped
# K=20 line, multi-view, deterministic-mode kernel stats, the W=8 rehearsals (RCCL modelled at 350 / 537
# GB/s with the tail in the all-to-all's group; the peer-store exchange)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fin6 gpurun_out/m
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rA > gpurun_out/fin6/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/fin6/tests.log | tail -12; exit 1; }
grep -E "passed|failed" gpurun_out/fin6/tests.log | tail -1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin6/smoke.log 2>&1 || { tail -5 gpurun_out/fin6/smoke.log; exit 1; }
tail -1 gpurun_out/fin6/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/m/bench_k20.log 2>&1 || { tail -5 gpurun_out/m/bench_k20.log; exit 1; }
timeout -k 10 300 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/m/bench_mv.log 2>&1 || { tail -5 gpurun_out/m/bench_mv.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/m/kt_det.log 2>&1 || { tail -5 gpurun_out/m/kt_det.log; exit 1; }
R="python3 bench.py --rehearse-world 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --fwd32-line 0 --parity 0"
for g in 350 537; do
  timeout -k 10 300 $R --link-gbps $g --plan-option TAIL_IN_A2A=1 > gpurun_out/m/rehearse_$g.log 2>&1 || { tail -5 gpurun_out/m/rehearse_$g.log; exit 1; }
done
timeout -k 10 300 $R --rehearse-comm peer > gpurun_out/m/rehearse_peer.log 2>&1 || { tail -5 gpurun_out/m/rehearse_peer.log; exit 1; }
timeout -k 10 300 $R --rehearse-comm copy > gpurun_out/m/rehearse_copy.log 2>&1 || { tail -5 gpurun_out/m/rehearse_copy.log; exit 1; }
for f in bench_k20 bench_mv rehearse_350 rehearse_537 rehearse_peer rehearse_copy; do python3 -c "import json;d=json.loads(open('gpurun_out/m/$f.log').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],d['value'])"; done
