#!/bin/bash
# GPU box: the whole -m gpu suite, smoke(), then the default bench line and a rocprofv3 kernel-trace
# summary of it.  Each GPU step under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
