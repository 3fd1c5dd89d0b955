#!/usr/bin/env bash
# Kernel traces of the bench's timed region at several K (tail-gap study); tools/tail_gaps.py reads them.
set -eu
mkdir -p gpurun_out/tg
export TMPDIR=/tmp
for k in ${KS:-10 20 40}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tg/k$k -o run \
    -- python3 bench.py --steps $k --warmup 10 --cpu-baseline 0 --fwd-only 0 --probes 0 ${EXTRA:-} > gpurun_out/tg/k$k.log 2>&1
  python3 tools/tail_gaps.py gpurun_out/tg/k$k/run_kernel_trace.csv $k | tee -a gpurun_out/tg/summary.txt
done
