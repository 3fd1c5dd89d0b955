#!/usr/bin/env bash
# bf16-wire data-parallel path on one GPU: kernel tests, per-rank compute rehearsals for
# W = 2/4/8, and a functional 2-rank gloo run of the full host schedule (both ranks on one GPU).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <seconds> <log> <cmd...>
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"; tail -2 "gpurun_out/$log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 300 wire_tests.log python -u -m pytest tests/test_gpu_wire.py -m gpu -x -v --timeout 120 --timeout-method thread
for W in 2 4 8; do
  run 300 rehearse_$W.log python bench.py --steps 100 --warmup 10 --cpu-baseline 0 --rehearse-world $W
done
run 400 gloo2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 3 --cpu-baseline 0 --backend gloo
