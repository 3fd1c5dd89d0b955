#!/bin/bash
# tight-row (parameter wire) SpMM: wire / DP parity tests, then the W=8 rehearsal's kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/u16t
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wire.py tests/test_gpu_dp_bow.py tests/test_gpu_graph.py > gpurun_out/u16t/tests.log 2>&1 || { tail -30 gpurun_out/u16t/tests.log; exit 1; }
tail -2 gpurun_out/u16t/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u16t/prof -o run -- python3 bench.py --rehearse-world 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --rehearse-comm model --link-gbps 1e9 --link-latency-us 0 --steps 56 --warmup 8 > gpurun_out/u16t/rehearse.log 2>&1 || { echo "rehearsal failed"; exit 1; }
python3 tools/kstats.py $(find gpurun_out/u16t/prof -name '*kernel_trace.csv' | head -1) 0 | grep -i "spmm\|adam\|gemm" 
bash tools/gpu_rehearse_w8.sh
