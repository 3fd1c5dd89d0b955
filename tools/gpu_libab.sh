#!/bin/bash
# A/B of library builds x plan options on the default bench.  Side builds: DSSM_BUILD_TAG=_<tag>
# [DSSM_EXTRA_CFLAGS=... DSSM_CSRC_DIR=<patched copy>] python -m dssm_amd.build -> libdssm_<tag>.so;
# "base" is the tree's own build.  Each variant is copied over dssm_amd/libdssm.so on the box: a bench
# line (K=200) per round, a rocprofv3 kernel-stats pass in round 1.
#   VARIANTS="base base:LAZY_ADAM=0 <tag>" ROUNDS=2 bash tools/gpu_libab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
cp dssm_amd/libdssm.so dssm_amd/libdssm_base.so
for r in $(seq 1 ${ROUNDS:-1}); do
for v in ${VARIANTS}; do
  tag=${v%%:*}; opt=""; [ "$tag" != "$v" ] && opt="--plan-option ${v#*:}"
  cp dssm_amd/libdssm_${tag}.so dssm_amd/libdssm.so
  name=$(echo "$v" | tr ':=' '__')
  timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0 $opt > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err || { echo "[$v] bench failed"; tail -5 gpurun_out/ab/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$name.json')); print('$v', d['ms_per_step'], d.get('kernels_ms'))"
  if [ "$r" = 1 ]; then
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof_$name -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0 $opt > gpurun_out/ab/prof_$name.log 2>&1 || { echo "[$v] rocprof failed"; exit 1; }
    python3 tools/kstats.py $(find gpurun_out/ab/prof_$name -name "*kernel_trace.csv" | head -1) 0 | head -9 > gpurun_out/ab/kstats_$name.txt
    cat gpurun_out/ab/kstats_$name.txt
  fi
done
done
cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so
