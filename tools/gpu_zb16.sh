#!/usr/bin/env bash
# ZB16 (bf16 hidden pre-BN activations, option off by default): the parity tests (default schedule and
# C2-zb16), then a bench A/B with the option on / off (alternating).  Each GPU step under its own limit.
set -eu
mkdir -p gpurun_out/zb
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2_bf16.py tests/test_gpu_dp_bow.py tests/test_gpu_wire.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/zb/tests.log 2>&1 || { grep -E "worst|Error|assert|FAIL" gpurun_out/zb/tests.log | head -30; tail -5 gpurun_out/zb/tests.log; exit 1; }
grep -E "worst" gpurun_out/zb/tests.log | head -20; tail -2 gpurun_out/zb/tests.log
B="--steps 400 --warmup 40 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0"
for r in 1 2 3; do
  for z in 1 0; do
    timeout -k 10 200 python3 bench.py $B --zb16 $z > gpurun_out/zb/b.json 2> gpurun_out/zb/b.err || { tail -20 gpurun_out/zb/b.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/zb/b.json').read().strip().splitlines()[-1]); print('zb16=$z', d['ms_per_step'], d['final_loss'], d['schedule'])"
  done
done
