#!/usr/bin/env bash
# Library A/B (tools/gpu_libab.sh) plus rocprofv3 kernel stats of each library.
set -u
bash tools/gpu_libab.sh "$@" || exit 1
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); mkdir -p gpurun_out/libst_$i
  DSSM_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/libst_$i -o run \
    -- python3 bench.py --steps 48 --warmup 8 --cpu-baseline 0 --fwd-only 0 > /dev/null 2>&1 || exit 1
done
