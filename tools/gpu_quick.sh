#!/usr/bin/env bash
# Quick GPU iteration: GPU tests, a bench line, a rocprofv3 kernel trace of a short bench.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
step() {  # step <seconds> <log> <cmd...>: stop the script at a crash / timeout
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then tail -20 "gpurun_out/$log"; echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
tail -3 gpurun_out/pytest_gpu.log
step 300 bench.log python bench.py --steps ${STEPS:-200} --warmup 20 --cpu-baseline 0 ${BENCH_ARGS:-}
tail -1 gpurun_out/bench.log | cut -c1-330
step 300 prof_bench.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --steps 48 --warmup 8 --cpu-baseline 0 ${BENCH_ARGS:-}
python tools/kstats.py gpurun_out/prof/run_kernel_trace.csv 16
