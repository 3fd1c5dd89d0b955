#!/usr/bin/env bash
# Functional rehearsal of the N>1 bench paths on ONE GPU: two ranks sharing the device over gloo
# (host-staged collectives: timings are meaningless), each exchange schedule / wire.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
port=29620
for args in "--wire bf16" "--wire fp32" "--dp-mode allreduce"; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 6 --warmup 2 --cpu-baseline 0 --backend gloo $args \
    > gpurun_out/dp.log 2>&1 || { echo "FAILED: $args"; tail -20 gpurun_out/dp.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/dp.log').read().strip().splitlines()[-1]); print('$args', d['config']['dp_exchange'], d['final_loss'], d['roofline']['kernel'], d['rooflines']['adam']['frac'])"
done
