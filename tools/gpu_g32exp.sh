#!/bin/bash
# fp32 tile experiments (diagnostics builds with timelines, wrong results): e1 no loads / staging in the
# chunk loop, e2 also no barrier, e3 also no LDS fragment reads (MFMA alone); e4 FRAGALL (correct)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g32exp
for v in g32tl e1 e2 e3 e4; do
  echo "== $v"
  DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_$v.so timeout -k 10 120 python tools/g32_timeline.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/g32exp/$v.txt || exit 1
done
cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1 || true
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python tools/dp_graph_noise.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/dp_graph_noise.txt
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python tools/mv_capture_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/mv_capture_probe.txt
