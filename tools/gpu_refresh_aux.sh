#!/usr/bin/env bash
# Refresh of the fp32 parity-mode and multi-view bench lines (default K / W; multi-view with its CPU baseline).
set -eu
mkdir -p gpurun_out/aux
timeout -k 10 300 python3 bench.py --dtype fp32 --cpu-baseline 0 > gpurun_out/aux/bench_fp32.log 2>&1
echo "fp32 ok"
timeout -k 10 400 python3 bench.py --model multiview > gpurun_out/aux/bench_multiview.log 2>&1
echo "mv ok"
