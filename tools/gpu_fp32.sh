#!/bin/bash
# fp32 parity mode: the GPU suite, the default bench line (its fp32_mode child) and the fp32 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f32/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/f32/gputests.log; exit 1; }
tail -2 gpurun_out/f32/gputests.log
timeout -k 10 400 python3 bench.py --cpu-baseline 0 > gpurun_out/f32/bench.json 2> gpurun_out/f32/bench.err || { echo "bench failed"; tail -20 gpurun_out/f32/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/f32/bench.json'));f=d.get('fp32_mode',{});print('bow', d['ms_per_step'], d['roofline']['frac'], 'fp32', f.get('ms_per_step'), f.get('roofline',{}).get('frac'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32/prof -o run -- python3 bench.py --dtype fp32 --cpu-baseline 0 --fp32-line 0 --det-line 0 --steps 50 --warmup 5 > gpurun_out/f32/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/f32/prof -name '*kernel_trace.csv' | head -1) 0
