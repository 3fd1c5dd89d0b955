#!/bin/bash
# round 6: the peer-store exchange's GPU tests, then the wire / DP regression tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6p
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 150 --timeout-method thread -rA > gpurun_out/r6p/peer.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/r6p/peer.log | head -40
[ $rc = 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_dp_bow.py tests/test_gpu_bench_dp.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r6p/wire.log 2>&1; rc=$?
tail -3 gpurun_out/r6p/wire.log
exit $rc
