#!/bin/bash
# round 4: RNN dW A/B + tests, multi-view / functional-op tests and bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="base dwold s64" ROUNDS=2 TESTED="base s64" bash tools/gpu_rnnab.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multiview.py tests/test_gpu_ops_bwd.py tests/test_gpu_api.py > gpurun_out/r4w.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4w.log; exit 1; }
tail -1 gpurun_out/r4w.log
timeout -k 10 400 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/r4w_mv.json 2> gpurun_out/r4w_mv.err || { echo "mv bench failed"; tail -20 gpurun_out/r4w_mv.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4w_mv.json'));print('mv', d['dtype'], d['ms_per_step'], d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'))"
