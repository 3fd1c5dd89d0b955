#!/bin/bash
# round 6: negative control of the peer self-test -- the side build with plain payload loads (_ld0, which
# read stale rows across processes) must fail the start-up self-test of the two-process IPC case
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6n
DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_ld0.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_peer.py::test_peer_world2_two_processes_ipc" -v --timeout 150 --timeout-method thread -rA > gpurun_out/r6n/neg.log 2>&1; rc=$?
echo "negative control rc=$rc (expected 1)"
grep -E "self-test failed|mismatching|PASSED|FAILED" gpurun_out/r6n/neg.log | head -8
[ $rc -le 1 ] || exit $rc
exit 0
