set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5a/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/r5a/tests.log; exit 1; }
tail -3 gpurun_out/r5a/tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5a/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/r5a/bench.log; exit 1; }
tail -1 gpurun_out/r5a/bench.log | cut -c1-600
