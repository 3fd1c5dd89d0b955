#!/bin/bash
# round 6: fp32 mode with W_l's pre-split planes (tests, kernel stats, bench lines); the sort variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6k
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c2_fp32.py tests/test_gpu_parity.py tests/test_gpu_fp32_schedule.py tests/test_gpu_deterministic.py tests/test_gpu_golden.py > gpurun_out/r6k/tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r6k/tests.log | head -20; tail -3 gpurun_out/r6k/tests.log; exit 1; }
tail -1 gpurun_out/r6k/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6k/kt_fp32 -o run -- python3 bench.py --dtype fp32 --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6k/kt_fp32.log 2>&1 || { tail -5 gpurun_out/r6k/kt_fp32.log; exit 1; }
for k in 20 200; do w=$([ $k = 20 ] && echo 5 || echo 20)
timeout -k 10 300 python3 bench.py --dtype fp32 --steps $k --warmup $w --cpu-baseline 0 > gpurun_out/r6k/bench_fp32_k$k.log 2>&1 || { tail -5 gpurun_out/r6k/bench_fp32_k$k.log; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r6k/bench_fp32_k$k.log').read().strip().splitlines()[-1]);print('fp32 K$k ms/step', d['ms_per_step'], d['roofline']['frac'], d['roofline']['bytes_per_launch'])"
done
for t in "" _s1 _s2 _s4 _s8 _s15; do
  DSSM_LIB_PATH=dssm_amd/libdssm$t.so timeout -k 10 120 python3 tools/sort_bench.py || exit 1
done
# the forward NT tile's B-panel share: a build that neither loads nor stages B (wrong results, timing only)
for t in "" _nob; do
  DSSM_LIB_PATH=dssm_amd/libdssm$t.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6k/kt_nt$t -o run -- python3 bench.py --steps 48 --warmup 8 --fp32-line 0 --det-line 0 --fwd-only 0 --cpu-baseline 0 > gpurun_out/r6k/kt_nt$t.log 2>&1 || { tail -5 gpurun_out/r6k/kt_nt$t.log; exit 1; }
  grep "k_gemm_nt_wk" gpurun_out/r6k/kt_nt$t/run_kernel_stats.csv | cut -d, -f1-6
done
timeout -k 10 120 python3 tools/ipc_probe.py || true
