#!/usr/bin/env bash
# One GPU-box session: smoke, GPU parity tests, short bench.  Stops at the first crash/timeout
# (exit >= 124 or signal) but keeps going after ordinary test failures (exit 1).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <seconds> <log> <cmd...>
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 400 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 900 pytest_gpu.log python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
run 600 bench.log python bench.py --steps ${STEPS:-100} --warmup 10 --cpu-baseline ${CPUB:-0}
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench.log
