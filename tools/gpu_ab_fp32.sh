#!/usr/bin/env bash
# fp32-mode and eval-forward A/B of two library builds, then the GPU suite on the default build.
set -u
mkdir -p gpurun_out
BENCH_ARGS="--dtype fp32" STEPS=100 ROUNDS=2 bash tools/gpu_libab.sh "$1" "$2" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
