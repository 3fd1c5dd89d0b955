#!/usr/bin/env bash
# Measurement set of the non-headline rows (profiles/<tag>_*_rnn / _mv): kernel-trace stats, PMC
# HBM traffic (FETCH_SIZE / WRITE_SIZE in separate passes) and, for the bf16 RNN, MFMA counters.
# Every GPU step under its own time limit; stops at the first failure.  Post-process on the CPU:
# tools/measure_post_aux.sh.
set -eu
mkdir -p gpurun_out/a
export TMPDIR=/tmp
for mdl in ${MODELS:-rnn multiview}; do
  B="python3 bench.py --model $mdl --cpu-baseline 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/a/kt_$mdl -o run \
    -- $B --steps 20 --warmup 3 > gpurun_out/a/kt_$mdl.log 2>&1
  echo "kt $mdl ok"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/a/pmc_$mdl/$c -o run \
      -- $B --steps 6 --warmup 2 --graph 0 --probes 0 > gpurun_out/a/pmc_${mdl}_$c.log 2>&1
    echo "pmc $mdl $c ok"
  done
  if [ $mdl = rnn ]; then
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
      --output-format csv -d gpurun_out/a/mfma_$mdl -o run \
      -- $B --steps 6 --warmup 2 --probes 0 > gpurun_out/a/mfma_$mdl.log 2>&1
    echo "mfma $mdl ok"
  fi
done
