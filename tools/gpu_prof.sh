#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps ${STEPS:-50} --warmup 5 --cpu-baseline 0 --fwd-only 0 > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
