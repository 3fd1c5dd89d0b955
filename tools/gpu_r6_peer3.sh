#!/bin/bash
# round 6: which side of the peer hand-off needs the system-scope accesses and which memory -- side builds (plain
# stores, plain loads, coarse-grained payload buffers), each through the two-process IPC test and the W=8 rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6p3
B="python3 bench.py --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 --fwd32-line 0 --parity 0 --steps 200 --warmup 20 --rehearse-world 8 --rehearse-comm peer"
for v in ${VARIANTS:-_c1 _c2}; do
  s=$v; [ "$v" = base ] && s=""; export DSSM_LIB_PATH=$GRAFT_REPO_ROOT/dssm_amd/libdssm$s.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_peer.py -v --timeout 150 --timeout-method thread -rA > gpurun_out/r6p3/peer$v.log 2>&1; rc=$?
  echo "variant $v tests rc=$rc"; grep -E "^(PASSED|FAILED)|differing per step|Mismatched" gpurun_out/r6p3/peer$v.log | head -12
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 $B > gpurun_out/r6p3/reh$v.json 2> gpurun_out/r6p3/reh$v.err; rc=$?
  [ $rc = 0 ] || { tail -3 gpurun_out/r6p3/reh$v.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r6p3/reh$v.json')); print('$v', d['ms_per_step'], d.get('dp_kernels_ms'))"
done
