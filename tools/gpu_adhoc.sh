set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_api.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wire.log 2>&1; tail -3 gpurun_out/pytest_wire.log
HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 120 python -u tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1; echo "probe rc=$?"; tail -20 gpurun_out/rccl_probe.log
