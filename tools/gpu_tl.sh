#!/usr/bin/env bash
# Diagnostics build with per-workgroup timelines (-DDSSM_WG_TL) + NT tile phase stamps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export DSSM_EXTRA_CFLAGS=-DDSSM_WG_TL
timeout -k 10 200 python -m dssm_amd.build --force > gpurun_out/tlbuild.log 2>&1 || exit $?
timeout -k 10 120 python tools/wg_timeline.py > gpurun_out/wgtl.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/wgtl.log
DSSM_DENSE=0 DSSM_NT_TIMING=1 timeout -k 10 120 python tools/dense_timing.py > gpurun_out/nttiming.log 2>&1
grep -v amdgpu.ids gpurun_out/nttiming.log
