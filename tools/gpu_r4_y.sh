#!/bin/bash
# multi-view: both towers' optimizer in one launch (pair) vs one launch per tower stream; tests; BoW
# Adam unchanged by the kernel-body refactor
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/y
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multiview.py tests/test_gpu_multiview_c5.py tests/test_gpu_ops_bwd.py tests/test_gpu_c2_bf16.py > gpurun_out/y/tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/y/tests.log; exit 1; }
tail -1 gpurun_out/y/tests.log
for r in 1 2; do
for v in 1 0; do
  DSSM_MV_ADAM_PAIR=$v timeout -k 10 300 python3 bench.py --model multiview --cpu-baseline 0 --fp32-line 0 > gpurun_out/y/mv_$v.json 2> gpurun_out/y/mv_$v.err || { echo "[$v] mv failed"; tail -5 gpurun_out/y/mv_$v.err; exit 1; }
  python3 -c "import json; a=json.load(open('gpurun_out/y/mv_$v.json')); print('pair=$v', a['ms_per_step'], a['roofline']['kernel'], a['roofline']['avg_ms'], a['roofline']['frac'])"
done
done
timeout -k 10 300 python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 > gpurun_out/y/bow.json 2> gpurun_out/y/bow.err || { echo "bow failed"; exit 1; }
python3 -c "import json; a=json.load(open('gpurun_out/y/bow.json')); print('bow', a['ms_per_step'], a['kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/y/prof -o run -- python3 bench.py --model multiview --steps 30 --warmup 3 --cpu-baseline 0 --fp32-line 0 > gpurun_out/y/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 tools/step_timeline.py $(find gpurun_out/y/prof -name "*kernel_trace.csv" | head -1)
