#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6f
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_wire.py -k "default_schedule" > gpurun_out/r6f/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|spread|passed|failed" gpurun_out/r6f/tests.log | tail -12
exit $rc
