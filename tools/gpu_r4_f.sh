#!/bin/bash
# multi-view fused W1 Adam: GPU tests, bench (bf16 + fp32 line), kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiview.py tests/test_gpu_multiview_c5.py tests/test_gpu_multiview_dp.py > gpurun_out/r4i_mv.log 2>&1 || { echo "multiview tests failed"; tail -60 gpurun_out/r4i_mv.log; exit 1; }
tail -1 gpurun_out/r4i_mv.log
for i in 1 2; do
timeout -k 10 400 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/r4i_mv_bench.json 2> gpurun_out/r4i_mv_bench.err || { echo "mv bench failed"; tail -20 gpurun_out/r4i_mv_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4i_mv_bench.json'));print('mv', d['dtype'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac'], d.get('fp32_mode',{}).get('ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i_mvprof -o run -- python3 bench.py --model multiview --steps 30 --warmup 3 --cpu-baseline 0 --fp32-line 0 > gpurun_out/r4i_mvprof.log 2>&1 || { echo "mv rocprof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/r4i_mvprof -name "*kernel_trace.csv" | head -1) 0 > gpurun_out/r4i_mv_kstats.txt 2>/dev/null; head -20 gpurun_out/r4i_mv_kstats.txt
