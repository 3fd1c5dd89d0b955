#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g32tl
export TMPDIR=/tmp
DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_g32tl.so timeout -k 10 120 python tools/g32_timeline.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g32tl/tl.txt
bash tools/gpu_r5b.sh > gpurun_out/g32tl/r5b.log 2>&1 || { tail -5 gpurun_out/g32tl/r5b.log; exit 1; }
head -14 gpurun_out/r5b/kstats.txt
