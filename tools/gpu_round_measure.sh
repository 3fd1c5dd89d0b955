#!/bin/bash
# a round's measurement set: tools/gpu_measure.sh (BoW bf16 + fp32: kernel stats, PMC traffic, MFMA,
# bench lines) and tools/gpu_measure_aux.sh for the RNN and multi-view rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"
DTYPES="bf16 fp32" bash tools/gpu_measure.sh || { echo "measure failed"; exit 1; }
MODELS="rnn multiview" bash tools/gpu_measure_aux.sh || { echo "aux failed"; exit 1; }
tail -1 gpurun_out/m/bench_bf16.log | cut -c1-300
