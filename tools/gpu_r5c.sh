#!/bin/bash
# round 5: the DP graph noise at the round-3 test's metric and the multi-view capture probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/dp_graph_noise.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/dp_graph_noise.txt || exit 1
timeout -k 10 600 python tools/mv_capture_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/mv_capture_probe.txt
