#!/bin/bash
# round-end rehearsal: the whole GPU suite, the default bench line and the other rows' lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fin
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/fin/gputests.log; exit 1; }
tail -2 gpurun_out/fin/gputests.log
timeout -k 10 400 python3 bench.py > gpurun_out/fin/bench.json 2> gpurun_out/fin/bench.err || { echo "bench failed"; tail -20 gpurun_out/fin/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fin/bench.json'));print('bow', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'), d.get('deterministic_mode',{}).get('ms_per_step'), d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/fin/bench_k20.json 2> gpurun_out/fin/bench_k20.err || { echo "bench k20 failed"; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fin/bench_k20.json'));print('bow k20', d['ms_per_step'], d['value'])"
timeout -k 10 400 python3 bench.py --model rnn > gpurun_out/fin/rnn.json 2> gpurun_out/fin/rnn.err || { echo "rnn bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fin/rnn.json'));print('rnn', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 python3 bench.py --model multiview > gpurun_out/fin/mv.json 2> gpurun_out/fin/mv.err || { echo "mv bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fin/mv.json'));print('mv', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'), d.get('cpu_baseline',{}).get('value'))"
