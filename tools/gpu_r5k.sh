#!/bin/bash
# 64-row forward tiles for the small-grid (last layer) forward: A/B against the previous rule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2_bf16.py tests/test_gpu_deterministic.py tests/test_gpu_graph.py tests/test_gpu_schedules.py tests/test_gpu_fused_stats.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
for v in "" _sg0 "" _sg0 "" _sg0; do
  DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm$v.so timeout -k 10 200 $B > $O/b$v.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$v.json'));print('variant [$v]',d['ms_per_step'])"
done
