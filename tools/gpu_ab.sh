#!/bin/bash
# A/B of the working tree's libdssm.so against side builds (libdssm<tag>.so for each argument,
# default _base), three alternations each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAGS=${*:-_base}
O=gpurun_out/ab; mkdir -p $O
B="python3 bench.py --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0 ${BENCH_ARGS:-}"
for r in $(seq ${ROUNDS:-3}); do
  for v in "" $TAGS; do
    DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm$v.so timeout -k 10 200 $B > $O/b$v.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b$v.json'));print('variant [$v]',d['ms_per_step'])"
  done
done
