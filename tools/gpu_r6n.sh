#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops_bwd.py -k csc_transpose tests/test_gpu_deterministic.py > gpurun_out/r6n_tests.log 2>&1 || { tail -20 gpurun_out/r6n_tests.log; exit 1; }
tail -1 gpurun_out/r6n_tests.log
for t in "" _s1 _s2 _s4 _s16; do
  DSSM_LIB_PATH=dssm_amd/libdssm$t.so timeout -k 10 120 python3 tools/sort_bench.py || exit 1
done
