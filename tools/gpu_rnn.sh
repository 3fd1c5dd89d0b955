#!/bin/bash
# RNN tower (config 4): the GPU suite, the bench line and one kernel-stats pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rnn
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rnn/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/rnn/gputests.log; exit 1; }
tail -2 gpurun_out/rnn/gputests.log
timeout -k 10 400 python3 bench.py --model rnn > gpurun_out/rnn/bench.json 2> gpurun_out/rnn/bench.err || { echo "rnn bench failed"; tail -20 gpurun_out/rnn/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/rnn/bench.json'));print('rnn', d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rnn/prof -o run -- python3 bench.py --model rnn --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/rnn/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/rnn/prof -name '*kernel_trace.csv' | head -1) 0 | head -16
