#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops_bwd.py tests/test_gpu_multiview.py tests/test_gpu_multiview_c5.py tests/test_gpu_rnn_bf16.py > gpurun_out/r4t.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r4t.log; exit 1; }
tail -3 gpurun_out/r4t.log
for shape in "6144 32" "4096 32" "4096 48" "6144 21"; do
timeout -k 10 120 python3 tools/adam_fn_bench.py $shape || exit 1
done
for i in 1 2; do
timeout -k 10 400 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/r4t_mv_bench.json 2> gpurun_out/r4t_mv_bench.err || { echo "mv bench failed"; tail -20 gpurun_out/r4t_mv_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4t_mv_bench.json'));print('mv', d['dtype'], d['ms_per_step'], d['roofline']['avg_ms'], d['roofline'].get('pair_span_ms'), d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'))"
timeout -k 10 400 python3 bench.py --model rnn --cpu-baseline 0 > gpurun_out/r4t_rnn_bench.json 2> gpurun_out/r4t_rnn_bench.err || { echo "rnn bench failed"; tail -20 gpurun_out/r4t_rnn_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4t_rnn_bench.json'));print('rnn', d['dtype'], d['ms_per_step'], d['roofline'].get('avg_ms'), d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4t_mvprof -o run -- python3 bench.py --model multiview --steps 30 --warmup 3 --cpu-baseline 0 --fp32-line 0 > gpurun_out/r4t_mvprof.log 2>&1 || { echo "mv rocprof failed"; exit 1; }
python3 tools/step_timeline.py $(find gpurun_out/r4t_mvprof -name "*kernel_trace.csv" | head -1)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4t_rnnprof -o run -- python3 bench.py --model rnn --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/r4t_rnnprof.log 2>&1 || { echo "rnn rocprof failed"; exit 1; }
python3 tools/step_timeline.py $(find gpurun_out/r4t_rnnprof -name "*kernel_trace.csv" | head -1) k_rnn_adam_advance
