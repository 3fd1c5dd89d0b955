#!/bin/bash
# the tight-row wire SpMM after the load fix: data-parallel tests, then the W = 8 rehearsal lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rh
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wire.py tests/test_gpu_dp_bow.py tests/test_gpu_graph.py tests/test_gpu_bench_dp.py > gpurun_out/rh/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/rh/tests.log; exit 1; }
tail -1 gpurun_out/rh/tests.log
bash tools/gpu_rehearse_w8.sh || exit 1
bash tools/gpu_rehearse_prof.sh | head -4
