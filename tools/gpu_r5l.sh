#!/bin/bash
# diagnostics: the fused statistics' fp64 atomics replaced by plain stores (wrong results): how
# much of the step the same-address atomic chains cost
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l; mkdir -p $O
B="python3 bench.py --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
for v in "" _noat "" _noat; do
  DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm$v.so timeout -k 10 200 $B > $O/b$v.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b$v.json'));print('variant [$v]',d['ms_per_step'])"
done
DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_noat.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --steps 50 --warmup 5 > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_trace.csv 0 > $O/kstats.txt; head -9 $O/kstats.txt
