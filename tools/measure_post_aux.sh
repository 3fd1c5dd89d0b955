#!/usr/bin/env bash
# CPU-side post-processing of tools/gpu_measure_aux.sh's gpurun_out/a into profiles/<tag>_*.
set -eu
TAG=${1:-r02}
for mdl in ${MODELS:-rnn multiview}; do
  if [ $mdl = rnn ]; then
    cp gpurun_out/a/kt_rnn/run_kernel_stats.csv profiles/${TAG}_rnn_kernel_stats.csv
    python3 tools/pmc_traffic.py gpurun_out/a/pmc_rnn profiles/${TAG}_traffic_rnn.json bf16 ids device rnn > /dev/null
    python3 tools/mfma_util.py gpurun_out/a/mfma_rnn profiles/${TAG}_rnn_kernel_stats.csv profiles/${TAG}_mfma_rnn.json bf16 rnn
  else
    # bench.py --model multiview runs the bf16 perf mode by default (round 4)
    cp gpurun_out/a/kt_multiview/run_kernel_stats.csv profiles/${TAG}_mv_kernel_stats.csv
    python3 tools/pmc_traffic.py gpurun_out/a/pmc_multiview profiles/${TAG}_traffic_mv_bf16.json bf16 zipf device multiview_bf16 > /dev/null
  fi
done
