#!/bin/bash
# TAIL_IN_A2A: the world-1 RCCL DP graph tests, and the W=8 rehearsal with the modelled links with the
# tail's all-reduce in the all-to-all's group
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_rccl.py tests/test_gpu_bench_dp.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --rehearse-world 8"
for g in 350 537; do
  for t in 0 1; do
    timeout -k 10 300 $B --link-gbps $g --plan-option TAIL_IN_A2A=$t > $O/r_${g}_$t.json 2> $O/r.err || { tail -5 $O/r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/r_${g}_$t.json'));print('W=8 $g GB/s TAIL_IN_A2A=$t',d['ms_per_step'])"
  done
done
