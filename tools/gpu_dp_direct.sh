#!/usr/bin/env bash
# DP wire checks and the one-GPU W = 8 rehearsal (compute only, device copies, modelled links).
set -eu
mkdir -p gpurun_out/dpd
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_rccl.py tests/test_gpu_dp_bow.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/dpd/tests.log 2>&1 || { tail -30 gpurun_out/dpd/tests.log; exit 1; }
tail -2 gpurun_out/dpd/tests.log
B="--steps 200 --warmup 20 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --rehearse-world 8"
for v in "--rehearse-comm model --link-gbps 1e9 --link-latency-us 0" "--rehearse-comm copy" "--rehearse-comm model"; do
  timeout -k 10 200 python3 bench.py $B $v > gpurun_out/dpd/b.json 2> gpurun_out/dpd/b.err || { tail -20 gpurun_out/dpd/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dpd/b.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('kernels_ms'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpd/kt -o run \
  -- python3 bench.py --steps 48 --warmup 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 \
  --rehearse-world 8 --rehearse-comm model --link-gbps 1e9 --link-latency-us 0 > /dev/null 2>&1
python3 tools/kstats.py gpurun_out/dpd/kt/run_kernel_trace.csv 14
