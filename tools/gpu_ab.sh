#!/usr/bin/env bash
# A/B: bench + rocprof stats for the default build and for env overrides given as args
# usage: bash tools/gpu_ab.sh "DSSM_SPLIT_FINALIZE=1" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "" "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python3 bench.py --steps ${STEPS:-200} --warmup 20 --cpu-baseline 0 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit $?
  echo "[$cfg] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); print(d['ms_per_step'], d['value'], d['kernels_ms'])")"
  if [ -n "$cfg" ]; then export $cfg; fi
  mkdir -p gpurun_out/prof_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$i -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline 0 > /dev/null 2>&1 || exit $?
  if [ -n "$cfg" ]; then unset ${cfg%%=*}; fi
done
