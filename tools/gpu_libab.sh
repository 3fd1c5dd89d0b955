#!/usr/bin/env bash
# A/B of library builds on the default bench, alternating runs to spread drift:
#   bash tools/gpu_libab.sh dssm_amd/libdssm_base.so dssm_amd/libdssm.so [...]
# ROUNDS (default 2) alternations; BENCH_ARGS extra bench flags.  Every run under its own limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in $(seq 1 "${ROUNDS:-2}"); do
  for lib in "$@"; do
    DSSM_LIB_PATH=$PWD/$lib timeout -k 10 200 python3 bench.py --steps ${STEPS:-400} --warmup 40 \
      --cpu-baseline 0 --fwd-only 0 ${BENCH_ARGS:-} > gpurun_out/libab.json 2> gpurun_out/libab.err || {
      echo "[$lib] failed rc=$?"; tail -5 gpurun_out/libab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/libab.json')); print('$lib', d['ms_per_step'], d['value'], d.get('kernels_ms'))"
  done
done
