#!/bin/bash
# the driver's round-end sequence at HEAD: smoke(), the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print('fp32_mode',d['fp32_mode']['ms_per_step'],'det',d.get('deterministic_mode',{}).get('ms_per_step'),'traffic',d['roofline']['traffic_source'])"
