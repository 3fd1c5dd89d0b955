#!/bin/bash
# round 6 measurement set at HEAD: GPU suite + smoke, kernel stats / PMC / MFMA for bf16 and fp32
# (tools/gpu_measure.sh), RNN + multi-view rows, the driver-shaped K=20 line, the deterministic
# line's kernel stats, the W=8 rehearsal at 350 / 537 GB/s with the tail in the all-to-all's group
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fin6 gpurun_out/m
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread -rA > gpurun_out/fin6/tests.log 2>&1 || { grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/fin6/tests.log | tail -12; exit 1; }
grep -E "passed|failed" gpurun_out/fin6/tests.log | tail -1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin6/smoke.log 2>&1 || { tail -5 gpurun_out/fin6/smoke.log; exit 1; }
tail -1 gpurun_out/fin6/smoke.log
bash tools/gpu_round_measure.sh || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/m/bench_k20.log 2>&1 || { tail -5 gpurun_out/m/bench_k20.log; exit 1; }
timeout -k 10 300 python3 bench.py --model multiview --cpu-baseline 0 > gpurun_out/m/bench_mv.log 2>&1 || { tail -5 gpurun_out/m/bench_mv.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m/kt_det -o run -- python3 bench.py --deterministic 1 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/m/kt_det.log 2>&1 || { tail -5 gpurun_out/m/kt_det.log; exit 1; }
for g in 350 537; do
  timeout -k 10 300 python3 bench.py --rehearse-world 8 --link-gbps $g --plan-option TAIL_IN_A2A=1 --cpu-baseline 0 --fp32-line 0 --det-line 0 --fwd-only 0 > gpurun_out/m/rehearse_$g.log 2>&1 || { tail -5 gpurun_out/m/rehearse_$g.log; exit 1; }
done
for f in bench_bf16 bench_fp32 bench_uniform bench_k20 bench_mv rehearse_350 rehearse_537; do python3 -c "import json;d=json.loads(open('gpurun_out/m/$f.log').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],d['value'])"; done
