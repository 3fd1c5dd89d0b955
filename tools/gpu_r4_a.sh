#!/bin/bash
# round 4: the bench-spawn tests, the full GPU suite, one default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_dp.py > gpurun_out/r4a_wire.log 2>&1 || { echo "bench tests failed"; tail -50 gpurun_out/r4a_wire.log; exit 1; }
tail -3 gpurun_out/r4a_wire.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4a_gpu.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/r4a_gpu.log; exit 1; }
tail -3 gpurun_out/r4a_gpu.log
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --fp32-line 0 --det-line 0 --cpu-baseline 0 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { echo "bench failed"; tail -30 gpurun_out/r4a_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r4a_bench.json'));print(d['ms_per_step'], d['kernels_ms'])"
