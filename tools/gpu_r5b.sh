#!/bin/bash
# round 5: the fp32 fused schedule's kernel stats (rocprofv3 kernel trace: per-kernel averages and
# one step's launch timeline, tools/kstats.py) and its bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 200 --warmup 20 --cpu-baseline 0 --fwd-only 0 > $O/bench_fp32.log 2>&1 || { tail -20 $O/bench_fp32.log; exit 1; }
tail -1 $O/bench_fp32.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --dtype fp32 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --steps 50 --warmup 5 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $(find $O/prof -name '*kernel_trace.csv' | head -1) 0 | tee $O/kstats.txt
