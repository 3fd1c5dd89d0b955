#!/usr/bin/env bash
# The DP graph tests (wire, RCCL, DP BoW, graphs) in one process, then the whole file again in a second
# process: the world-1 graph-vs-eager cases must hold in both.  Each step under its own limit.
set -eu
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_rccl.py tests/test_gpu_dp_bow.py tests/test_gpu_graph.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/wire_rep$r.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/wire_rep$r.log | head; exit 1; }
  tail -1 gpurun_out/wire_rep$r.log
done
