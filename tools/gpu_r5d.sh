#!/bin/bash
# round 5: the whole GPU suite after the fp32 tile changes + the three-stream multi-view option,
# the driver-shaped bench line (fp32_mode beside it), and multi-view two- vs three-stream step time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed" $O/tests.log | tail -15; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bf16',d['ms_per_step'],'fp32',d.get('fp32_mode',{}).get('ms_per_step'),'det',d.get('deterministic',{}).get('ms_per_step') if isinstance(d.get('deterministic'),dict) else None)"
for cs in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --model multiview --mv-csc-stream $cs --cpu-baseline 0 --fp32-line 0 > $O/mv_$cs.json 2>> $O/mv.err || { tail -20 $O/mv.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/mv_$cs.json'));print('mv csc_stream $cs',d['ms_per_step'],d['config']['csc_stream'])"
done
