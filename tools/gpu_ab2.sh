#!/usr/bin/env bash
# A/B of bench launch modes: each arg is "ENV=.. --bench-flags" (env part optional, ';'-separated)
# usage: bash tools/gpu_ab2.sh "--graph 0" "--graph 1 --probes 0" "DSSM_CSC_INLINE=1;--graph 1"
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""; flags="$spec"
  if [[ "$spec" == *";"* ]]; then envs="${spec%%;*}"; flags="${spec#*;}"; fi
  env $envs timeout -k 10 300 python3 bench.py --steps ${STEPS:-300} --warmup 20 --cpu-baseline 0 $flags > gpurun_out/ab2_$i.json 2> gpurun_out/ab2_$i.err || exit $?
  echo "[$spec] $(python3 -c "import json; d=json.load(open('gpurun_out/ab2_$i.json')); print(d['ms_per_step'], d['value'], d['kernels_ms'])")"
done
