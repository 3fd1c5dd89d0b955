#!/bin/bash
# round 6: deterministic mode's write-through hand-offs: the deterministic tests, then its kernel stats and K=20 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6i
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_deterministic.py tests/test_gpu_graph.py tests/test_gpu_wire.py tests/test_gpu_c2_fp32.py tests/test_gpu_ops_bwd.py > gpurun_out/r6i/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r6i/tests.log | head -20; tail -3 gpurun_out/r6i/tests.log; exit 1; }
tail -1 gpurun_out/r6i/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6i/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6i/kt_det.log 2>&1 || { tail -5 gpurun_out/r6i/kt_det.log; exit 1; }
timeout -k 10 300 python3 bench.py --deterministic 1 --steps 20 --warmup 5 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6i/bench_det_k20.log 2>&1 || { tail -5 gpurun_out/r6i/bench_det_k20.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6i/bench_det_k20.log').read().strip().splitlines()[-1]);print('det K20 ms/step', d['ms_per_step'])"
