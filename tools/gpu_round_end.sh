#!/usr/bin/env bash
# Round-end set: the whole -m gpu suite, smoke(), rocprofv3 kernel stats of the headline run, the
# default bench line (CPU baseline, fp32 / deterministic lines), the driver-shaped K=20 / W=5 line and
# the W=8 data-parallel rehearsal.  Every GPU step under its own limit; the first failure ends it.
set -eu
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 \
  || { tail -30 gpurun_out/fin/gputests.log; exit 1; }
tail -2 gpurun_out/fin/gputests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1
tail -1 gpurun_out/fin/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/kt -o run \
  -- python3 bench.py --steps 48 --warmup 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 > gpurun_out/fin/kt.log 2>&1
echo "kt ok"
timeout -k 10 400 python3 bench.py > gpurun_out/fin/bench_bf16.json 2> gpurun_out/fin/bench_bf16.err
echo "bench ok"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/fin/bench_bf16_k20.json 2> gpurun_out/fin/bench_bf16_k20.err
echo "k20 ok"
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 \
  --rehearse-world 8 > gpurun_out/fin/rehearse_w8.json 2> gpurun_out/fin/rehearse_w8.err
echo "rehearse ok"
for f in bench_bf16 bench_bf16_k20 rehearse_w8; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], d['roofline']['frac'], (d.get('fp32_mode') or {}).get('ms_per_step'), (d.get('deterministic_mode') or {}).get('ms_per_step'))" gpurun_out/fin/$f.json $f
done
