#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/u16t
export TMPDIR=/tmp
cp dssm_amd/libdssm.so dssm_amd/libdssm_base.so
for v in base plain; do
  cp dssm_amd/libdssm_$v.so dssm_amd/libdssm.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u16t/prof_$v -o run -- python3 bench.py --rehearse-world 8 --cpu-baseline 0 --fp32-line 0 --det-line 0 --rehearse-comm model --link-gbps 1e9 --link-latency-us 0 --steps 56 --warmup 8 > gpurun_out/u16t/$v.log 2>&1 || { echo "failed $v"; cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so; exit 1; }
  echo "$v $(python3 tools/kstats.py $(find gpurun_out/u16t/prof_$v -name '*kernel_trace.csv' | head -1) 0 | grep spmm_scan)"
done
cp dssm_amd/libdssm_base.so dssm_amd/libdssm.so
