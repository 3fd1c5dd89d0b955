#!/usr/bin/env bash
# CPU-side post-processing of tools/gpu_measure.sh's gpurun_out/m into profiles/<tag>_*.
set -eu
TAG=${1:-r02}
for dt in ${DTYPES:-bf16 fp32}; do
  sfx=$([ $dt = bf16 ] && echo "" || echo "_$dt")
  cp gpurun_out/m/kt_$dt/run_kernel_stats.csv profiles/${TAG}_kernel_stats$sfx.csv
  python3 tools/pmc_traffic.py gpurun_out/m/pmc_$dt profiles/${TAG}_traffic$sfx.json $dt zipf device > /dev/null
  python3 tools/mfma_util.py gpurun_out/m/mfma_$dt profiles/${TAG}_kernel_stats$sfx.csv profiles/${TAG}_mfma$sfx.json $dt
done
