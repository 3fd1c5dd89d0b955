#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6h
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops_bwd.py -k csc_transpose tests/test_gpu_deterministic.py tests/test_gpu_graph.py > gpurun_out/r6h/tests.log 2>&1 || { tail -30 gpurun_out/r6h/tests.log; exit 1; }
tail -1 gpurun_out/r6h/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6h/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6h/kt_det.log 2>&1 || { tail -5 gpurun_out/r6h/kt_det.log; exit 1; }
python3 tools/kstats.py gpurun_out/r6h/kt_det/run_kernel_stats.csv 2>/dev/null | head -12 || true
grep -i sort gpurun_out/r6h/kt_det/run_kernel_stats.csv | cut -d, -f1-8
timeout -k 10 300 python3 bench.py --deterministic 1 --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6h/bench_det_k20.log 2>&1 || { tail -5 gpurun_out/r6h/bench_det_k20.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6h/bench_det_k20.log').read().strip().splitlines()[-1]);print('det K20 ms/step', d['ms_per_step'])"
