#!/usr/bin/env bash
# Headline bench of side trees under _bisect/<name>/ (each with its own built library) beside the
# current tree, alternating ROUNDS times (CUR_ARGS: flags for the current tree only).  Every run under its own limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$PWD
for r in $(seq 1 "${ROUNDS:-2}"); do
  for t in "$@"; do
    if [ "$t" = "." ]; then d=$ROOT; else d=$ROOT/_bisect/$t; fi
    (cd "$d" && timeout -k 10 200 python3 bench.py --steps ${STEPS:-200} --warmup ${WARMUP:-20} --cpu-baseline 0 \
      --fwd-only 0 --fp32-line 0 ${BENCH_ARGS:-} $( [ "$t" = "." ] && echo "${CUR_ARGS:-}" ) > $ROOT/gpurun_out/bisect.json 2> $ROOT/gpurun_out/bisect.err) || {
      echo "[$t] failed"; tail -5 gpurun_out/bisect.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bisect.json').read().splitlines()[-1]); print('$t', d['ms_per_step'], d['kernels_ms'])"
  done
done
