#!/bin/bash
# round 4: lazy-Adam parity + the A/B of LAZY_ADAM on the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lazy.py tests/test_gpu_graph.py tests/test_gpu_c2_bf16.py > gpurun_out/r4c_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r4c_tests.log; exit 1; }
tail -2 gpurun_out/r4c_tests.log
VARIANTS="base base:LAZY_ADAM=0" ROUNDS=${ROUNDS:-3} bash tools/gpu_libab.sh 2>&1 | grep -v "BrokenPipe\|Traceback\|File \|main(\|print("
