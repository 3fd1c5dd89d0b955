#!/bin/bash
# RNN (config 4) A/B of library builds: the bf16 parity tests on the listed builds, then a bench line
# per build per round and one kernel-stats pass.  VARIANTS="base dwold s64" ROUNDS=2 TESTED="base s64"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rab
export TMPDIR=/tmp
cp dssm_amd/libdssm.so dssm_amd/libdssm_base.so
for v in ${TESTED:-base}; do
  cp dssm_amd/libdssm_$v.so dssm_amd/libdssm.so
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rnn_bf16.py > gpurun_out/rab/test_$v.log 2>&1 || { echo "[$v] rnn tests failed"; tail -40 gpurun_out/rab/test_$v.log; cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/rab/test_$v.log)"
done
for r in $(seq 1 ${ROUNDS:-1}); do
for v in ${VARIANTS}; do
  cp dssm_amd/libdssm_$v.so dssm_amd/libdssm.so
  timeout -k 10 300 python3 bench.py --model rnn --steps 100 --cpu-baseline 0 > gpurun_out/rab/$v.json 2> gpurun_out/rab/$v.err || { echo "[$v] bench failed"; tail -5 gpurun_out/rab/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rab/$v.json')); print('$v', d['ms_per_step'])"
  if [ "$r" = 1 ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rab/prof_$v -o run -- python3 bench.py --model rnn --steps 20 --warmup 3 --cpu-baseline 0 > gpurun_out/rab/prof_$v.log 2>&1 || { echo "[$v] rocprof failed"; exit 1; }
    python3 tools/kstats.py $(find gpurun_out/rab/prof_$v -name "*kernel_trace.csv" | head -1) 0 | head -8
  fi
done
done
cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so
