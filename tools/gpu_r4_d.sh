#!/bin/bash
# round 4: multi-view bf16 mode: config-5 parity (fp32 + bf16), the GPU suite, the multiview bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_multiview_c5.py > gpurun_out/r4d_mv.log 2>&1 || { echo "multiview tests failed"; tail -60 gpurun_out/r4d_mv.log; exit 1; }
grep -E "config-5|PASS|FAIL" gpurun_out/r4d_mv.log | tail -12
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4d_gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r4d_gpu.log; exit 1; }
tail -2 gpurun_out/r4d_gpu.log
timeout -k 10 400 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/r4d_mv_bench.json 2> gpurun_out/r4d_mv_bench.err || { echo "mv bench failed"; tail -20 gpurun_out/r4d_mv_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4d_mv_bench.json'));print('mv', d['dtype'], d['ms_per_step'], d['roofline']['avg_ms'], d.get('fp32_mode',{}).get('ms_per_step'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d_mvprof -o run -- python3 bench.py --model multiview --steps 30 --warmup 3 --cpu-baseline 0 --fp32-line 0 > gpurun_out/r4d_mvprof.log 2>&1 || { echo "mv rocprof failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/r4d_mvprof -name "*kernel_trace.csv" | head -1) 0 > gpurun_out/r4d_mv_kstats.txt 2>/dev/null; head -16 gpurun_out/r4d_mv_kstats.txt
