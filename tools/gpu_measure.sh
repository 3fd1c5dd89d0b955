#!/usr/bin/env bash
# One round's measurement set (profiles/<tag>_*): kernel-trace stats, PMC HBM traffic
# (FETCH_SIZE / WRITE_SIZE in separate passes) and MFMA counters, for the bf16 headline and the
# fp32 parity-mode workloads, plus the bench lines.  Every GPU step under its own time limit; the
# script stops at the first failure.  Post-process on the CPU: tools/measure_post.sh.
set -eu
mkdir -p gpurun_out/m
export TMPDIR=/tmp
B="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0"
for dt in ${DTYPES:-bf16 fp32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m/kt_$dt -o run \
    -- $B --dtype $dt --steps 48 --warmup 8 --fwd-only 0 > gpurun_out/m/kt_$dt.log 2>&1
  echo "kt $dt ok"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/m/pmc_$dt/$c -o run \
      -- $B --dtype $dt --steps 16 --warmup 3 --graph 0 --probes 0 --fwd-only 0 > gpurun_out/m/pmc_${dt}_$c.log 2>&1
    echo "pmc $dt $c ok"
  done
  # fp32: the split tiles run bf16 MFMAs (csrc/g32.h), the exact build f32 ones: count both
  M=SQ_INSTS_VALU_MFMA_MOPS_BF16; [ $dt = fp32 ] && M="SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16"
  timeout -k 10 300 rocprofv3 --pmc $M SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    -d gpurun_out/m/mfma_$dt -o run \
    -- $B --dtype $dt --steps 16 --warmup 3 --graph 0 --probes 0 --fwd-only 0 > gpurun_out/m/mfma_$dt.log 2>&1
  echo "mfma $dt ok"
done
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python3 bench.py > gpurun_out/m/bench_bf16.log 2>&1
  timeout -k 10 300 python3 bench.py --dtype fp32 --cpu-baseline 0 > gpurun_out/m/bench_fp32.log 2>&1
  timeout -k 10 300 python3 bench.py --columns uniform --cpu-baseline 0 > gpurun_out/m/bench_uniform.log 2>&1
  tail -1 gpurun_out/m/bench_bf16.log | cut -c1-400
fi
