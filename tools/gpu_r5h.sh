#!/bin/bash
# round 5: the whole GPU suite (sparse exchange, folded BN backward, split fp32 tiles), then the
# N=2 gloo bench with its three legs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -40; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0"
for g in 350 537; do
  timeout -k 10 300 $B --rehearse-world 8 --link-gbps $g > $O/rehearse_$g.json 2> $O/rehearse.err || { tail -5 $O/rehearse.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/rehearse_$g.json'));print('rehearse W=8 $g GB/s',d['ms_per_step'],d.get('dp_kernels_ms'))"
done
timeout -k 10 300 $B --rehearse-world 8 --rehearse-comm copy > $O/rehearse_copy.json 2>> $O/rehearse.err || { tail -5 $O/rehearse.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rehearse_copy.json'));print('rehearse W=8 compute share (copies)',d['ms_per_step'])"
