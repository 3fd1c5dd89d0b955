#!/bin/bash
# multi-view row: the GPU suite, the functional dense backward alone, the multi-view bench line and kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mv
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mv/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/mv/gputests.log; exit 1; }
tail -2 gpurun_out/mv/gputests.log
timeout -k 10 120 python3 tools/dense_bwd_bench.py || exit 1
timeout -k 10 400 python3 bench.py --model multiview > gpurun_out/mv/bench.json 2> gpurun_out/mv/bench.err || { echo "mv bench failed"; tail -20 gpurun_out/mv/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/mv/bench.json'));print('mv', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mv/prof -o run -- python3 bench.py --model multiview --steps 30 --warmup 3 --cpu-baseline 0 --fp32-line 0 > gpurun_out/mv/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/mv/prof -name '*kernel_trace.csv' | head -1) 0 | head -14
