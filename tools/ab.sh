#!/usr/bin/env bash
# A/B of env knobs on the default bench: tools/ab.sh "VAR=1" "VAR=0 OTHER=2" ...
set -u
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 40 --cpu-baseline 0 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], d['kernels_ms'])"
done
