#!/usr/bin/env bash
# Multi-view (config 5) A/B of two library builds, then the multi-view / fp32 GPU tests on the default build.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for lib in "$1" "$2"; do
    DSSM_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 bench.py --model multiview --steps 100 --warmup 10 --cpu-baseline 0 \
      > gpurun_out/mvab.json 2> gpurun_out/mvab.err || { echo "[$lib] failed"; tail -5 gpurun_out/mvab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/mvab.json').read().strip().splitlines()[-1]); print('$lib', d['ms_per_step'], d['value'])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
