#!/bin/bash
# round 6: the whole GPU suite and the smoke, as the driver runs them at round end
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6s
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rA > gpurun_out/r6s/tests.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/r6s/tests.log | tail -15
grep -E "updates within|parameters within" gpurun_out/r6s/tests.log | head -8
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6s/smoke.log 2>&1 || { tail -5 gpurun_out/r6s/smoke.log; exit 1; }
tail -2 gpurun_out/r6s/smoke.log
