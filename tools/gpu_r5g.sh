#!/bin/bash
# fp32 split tiles after the address clean-up: fp32 GPU tests, bench, timeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c2_fp32.py tests/test_gpu_parity.py tests/test_gpu_fp32_schedule.py tests/test_gpu_deterministic.py tests/test_gpu_fused_stats.py tests/test_gpu_graph.py tests/test_gpu_golden.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed|^E  " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --dtype fp32 --cpu-baseline 0 --fwd-only 0 --fp32-line 0 --det-line 0"
for i in 1 2; do timeout -k 10 200 $B > $O/b$i.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }; python3 -c "import json;d=json.load(open('$O/b$i.json'));print('fp32 K=200',d['ms_per_step'])"; done
DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm_g32tl.so timeout -k 10 120 python tools/g32_timeline.py 2>&1 | grep -v amdgpu.ids | tee $O/tl.txt
