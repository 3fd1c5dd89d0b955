#!/bin/bash
# GPU box: data-parallel wire / RCCL tests, then one-GPU rehearsals of the 8-rank step graph.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r3dp}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_rccl.py tests/test_gpu_dp_bow.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="--steps 20 --warmup 5 --fwd-only 0 --cpu-baseline 0 --fp32-line 0"
: > gpurun_out/${T}_rehearse.txt
while read -r args; do
  [ -z "$args" ] && continue
  timeout -k 10 200 python bench.py $B $args > gpurun_out/${T}_tmp.json 2>> gpurun_out/${T}_bench.err || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/${T}_tmp.json')); print(sys.argv[1], '->', d['ms_per_step'], 'ms/step', d['kernels_ms'], d['final_loss'])" "$args" | tee -a gpurun_out/${T}_rehearse.txt
done <<'LIST'
--rehearse-world 8 --rehearse-comm model --link-gbps 1e9 --link-latency-us 0
--rehearse-world 8 --rehearse-comm model
--rehearse-world 8 --rehearse-comm copy
--rehearse-world 2 --rehearse-comm model
LIST
