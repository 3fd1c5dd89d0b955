#!/usr/bin/env bash
# Multi-view (config 5): GPU tests, then the bench line (one-graph timed region, twice) and kernel stats.
set -eu
mkdir -p gpurun_out/mv
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiview.py tests/test_gpu_multiview_c5.py tests/test_gpu_multiview_dp.py \
  tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_rnn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mv/tests.log 2>&1 \
  || { tail -30 gpurun_out/mv/tests.log; exit 1; }
tail -2 gpurun_out/mv/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model multiview > gpurun_out/mv/b$r.json 2> gpurun_out/mv/b.err || { tail -20 gpurun_out/mv/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mv/b$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d.get('roofline',{}).get('frac'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mv/kt -o run \
  -- python3 bench.py --model multiview --cpu-baseline 0 --steps 30 --warmup 5 > /dev/null 2>&1
python3 tools/kstats.py gpurun_out/mv/kt/run_kernel_trace.csv 14
