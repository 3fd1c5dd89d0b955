#!/bin/bash
# round 5: the split-bf16 fp32 tiles and the folded last-layer BN backward (bf16): the whole GPU
# suite, bench lines (A/B of BNB_IN_PAIR), kernel stats of both dtypes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -40; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
timeout -k 10 300 $B --dtype fp32 > $O/bench_fp32.json 2> $O/bench_fp32.err || { tail -20 $O/bench_fp32.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fp32.json'));print('fp32 K=200',d['ms_per_step'],d['roofline']['frac'])"
for v in 1 0 1 0; do
  timeout -k 10 300 $B --plan-option BNB_IN_PAIR=$v > $O/bench_bf16_bnb$v.json 2> $O/bench_bf16.err || { tail -20 $O/bench_bf16.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_bf16_bnb$v.json'));print('bf16 K=200 BNB_IN_PAIR=$v',d['ms_per_step'],d['roofline']['frac'])"
done
for dt in fp32 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$dt -o run -- python3 bench.py --dtype $dt --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --steps 50 --warmup 5 > $O/prof_$dt.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof_$dt.log; exit 1; }
  python3 tools/kstats.py $O/prof_$dt/run_kernel_trace.csv 0 > $O/kstats_$dt.txt; head -12 $O/kstats_$dt.txt
done
