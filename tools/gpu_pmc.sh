#!/usr/bin/env bash
# HBM traffic per kernel from rocprofv3 PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in separate passes (they do not fit one pass), no trace domains.  Parsed by
# tools/pmc_traffic.py into profiles/<tag>_traffic.json, which bench.py reads for "traffic".
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc/$c -o run \
    -- python3 bench.py --steps ${STEPS:-20} --warmup 3 --cpu-baseline 0 --graph 0 --probes 0 --fwd-only 0 ${BENCH_ARGS:-} \
    > gpurun_out/pmc/$c.log 2>&1 || exit $?
done
find gpurun_out/pmc -name "*counter_collection*"
