#!/bin/bash
# round 5: fp32 split vs exact tiles end to end against the float64 oracle (per layer / gradient),
# then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/diag_fp32_split.py both > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
