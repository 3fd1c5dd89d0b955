#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops_bwd.py > gpurun_out/r4t.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r4t.log; exit 1; }
tail -3 gpurun_out/r4t.log
for shape in "6144 32" "4096 32" "4096 48" "6144 21"; do
timeout -k 10 120 python3 tools/adam_fn_bench.py $shape || exit 1
done
