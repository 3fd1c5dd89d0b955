#!/bin/bash
# fp32 split tiles: A/B of build variants (WN=4: 8 waves of 32x16; DEPTH=2) on the fp32 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g32ab; mkdir -p $O
B="python3 bench.py --dtype fp32 --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
for v in "" _wn4 _d2 "" _wn4 _d2; do
  DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm$v.so timeout -k 10 200 $B > $O/b$v.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$v.json'));print('variant [$v]',d['ms_per_step'])"
done
