set -eu
mkdir -p gpurun_out
export TMPDIR=/tmp
L=dssm_amd/libdssm
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_rank.log 2>&1 || { tail -30 gpurun_out/pytest_rank.log; exit 1; }
tail -1 gpurun_out/pytest_rank.log
STEPS=400 bash tools/ab.sh "DSSM_LIB_PATH=$L.so" "DSSM_LIB_PATH=${L}_r32.so" "DSSM_LIB_PATH=${L}_r48.so" "DSSM_LIB_PATH=$L.so" "DSSM_LIB_PATH=${L}_r32.so" "DSSM_LIB_PATH=${L}_r48.so"
