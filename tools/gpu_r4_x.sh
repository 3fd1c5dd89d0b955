#!/bin/bash
# A/B: the functional cosine's in-kernel loss finalize (base) vs the separate finalize launch (nofin),
# on the multi-view and RNN benches, alternating; then the RNN tests on base
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/x
cp dssm_amd/libdssm.so dssm_amd/libdssm_base.so
for r in 1 2; do
for v in base nofin; do
  cp dssm_amd/libdssm_$v.so dssm_amd/libdssm.so
  timeout -k 10 300 python3 bench.py --model multiview --cpu-baseline 0 --fp32-line 0 > gpurun_out/x/mv_$v.json 2> gpurun_out/x/mv_$v.err || { echo "[$v] mv failed"; tail -5 gpurun_out/x/mv_$v.err; cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so; exit 1; }
  timeout -k 10 300 python3 bench.py --model rnn --cpu-baseline 0 --steps 100 > gpurun_out/x/rnn_$v.json 2> gpurun_out/x/rnn_$v.err || { echo "[$v] rnn failed"; tail -5 gpurun_out/x/rnn_$v.err; cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so; exit 1; }
  python3 -c "import json; a=json.load(open('gpurun_out/x/mv_$v.json')); b=json.load(open('gpurun_out/x/rnn_$v.json')); print('$v', 'mv', a['ms_per_step'], 'rnn', b['ms_per_step'])"
done
done
cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rnn_bf16.py tests/test_gpu_rnn.py > gpurun_out/x/rnn_tests.log 2>&1 || { echo "rnn tests failed"; tail -30 gpurun_out/x/rnn_tests.log; exit 1; }
tail -1 gpurun_out/x/rnn_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x/prof_rnn -o run -- python3 bench.py --model rnn --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/x/prof_rnn.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/step_timeline.py $(find gpurun_out/x/prof_rnn -name "*kernel_trace.csv" | head -1) k_rnn_adam
