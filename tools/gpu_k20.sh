#!/usr/bin/env bash
# K = 20 fixed-cost study: the driver-shaped region (W = 5) against a longer warm-up, a host idle or a
# dense matmul load before the warm-up, and K = 200.  Each run under its own limit; the first failure
# ends the script.
set -eu
mkdir -p gpurun_out/k20
B="--cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0"
run() {  # run <tag> <args...>
  local tag=$1; shift
  timeout -k 10 120 python3 bench.py $B "$@" > gpurun_out/k20/$tag.json 2> gpurun_out/k20/$tag.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/k20/$tag.json $tag
}
for r in 1 2; do
  run w5_$r --steps 20 --warmup 5
  run busy50ms_$r --steps 20 --warmup 5 --busy-before-warmup 0.05
  run busy500ms_$r --steps 20 --warmup 5 --busy-before-warmup 0.5
  run w200_$r --steps 20 --warmup 200
  run k200_$r --steps 200 --warmup 20
done
