#!/bin/bash
# timeline of the split fp32 tiles (diagnostics build libdssm_g32tl.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g32tl2
export TMPDIR=/tmp
DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_g32tl.so timeout -k 10 120 python tools/g32_timeline.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g32tl2/tl.txt
