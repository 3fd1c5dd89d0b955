#!/bin/bash
# both hidden layers' BN backward folded into their pairs (BNB_IN_PAIR): bf16 GPU tests, A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -40; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
for v in 1 0 1 0; do
  timeout -k 10 300 $B --plan-option BNB_IN_PAIR=$v > $O/b$v.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$v.json'));print('bf16 K=200 BNB_IN_PAIR=$v',d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --steps 50 --warmup 5 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_trace.csv 0 > $O/kstats.txt; head -11 $O/kstats.txt
