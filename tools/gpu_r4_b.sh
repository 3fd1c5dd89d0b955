#!/bin/bash
# round 4: row-panel NT + lazy Adam + csc_col skip: parity of the fused path, bench, rocprof stats,
# then the full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lazy.py tests/test_gpu_c2_bf16.py tests/test_gpu_graph.py tests/test_gpu_fused_stats.py > gpurun_out/r4b_c2.log 2>&1 || { echo "parity tests failed"; tail -60 gpurun_out/r4b_c2.log; exit 1; }
tail -2 gpurun_out/r4b_c2.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --fp32-line 0 --det-line 0 --cpu-baseline 0 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || { echo "bench failed"; tail -30 gpurun_out/r4b_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4b_bench.json'));print('K200', d['ms_per_step'], d['kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_prof -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0 > gpurun_out/r4b_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/r4b_prof.log; exit 1; }
python tools/kstats.py $(find gpurun_out/r4b_prof -name "*kernel_trace.csv" | head -1) 14 > gpurun_out/r4b_kstats.txt
head -20 gpurun_out/r4b_kstats.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4b_gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r4b_gpu.log; exit 1; }
tail -3 gpurun_out/r4b_gpu.log
