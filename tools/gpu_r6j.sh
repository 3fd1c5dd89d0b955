#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for t in "" _s1 _s2 _s4 _s8 _s15; do
  DSSM_LIB_PATH=dssm_amd/libdssm$t.so timeout -k 10 120 python3 tools/sort_bench.py || exit 1
done
