#!/bin/bash
# BoW headline A/B of side builds: bash tools/gpu_ab_bow.sh base tagA tagB ...
# (dssm_amd/libdssm_<tag>.so built beforehand with DSSM_BUILD_TAG; "base" = the in-tree build).
# Per variant: the bench line (K = 200) and a rocprofv3 kernel-stats pass (K = 50).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
cp dssm_amd/libdssm.so dssm_amd/libdssm_base.so
restore() { cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so; }
for v in "$@"; do
  cp dssm_amd/libdssm_$v.so dssm_amd/libdssm.so
  timeout -k 10 300 python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { echo "[$v] bench failed"; tail -5 gpurun_out/ab/$v.err; restore; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.json')); r=d['roofline']; print('[$v]', d['ms_per_step'], 'adam', r.get('achieved'), r.get('frac'), d.get('kernels_ms'))" | cut -c1-400
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$v -o run -- python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --steps 50 --warmup 5 > gpurun_out/ab/prof_$v.log 2>&1 || { echo "[$v] rocprof failed"; restore; exit 1; }
  python3 tools/kstats.py $(find gpurun_out/ab/prof_$v -name '*kernel_trace.csv' | head -1) 0 | head -12
done
restore
