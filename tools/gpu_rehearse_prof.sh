#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rh
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rh/prof -o run -- python3 bench.py --rehearse-world 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --rehearse-comm model --link-gbps 1e9 --link-latency-us 0 --steps 56 --warmup 8 > gpurun_out/rh/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/rh/prof.log; exit 1; }
python3 tools/kstats.py $(find gpurun_out/rh/prof -name "*kernel_trace.csv" | head -1) 30 > gpurun_out/rh/kstats.txt
cat gpurun_out/rh/kstats.txt
