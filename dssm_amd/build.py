"""Build libdssm.so in-tree: hipcc --offload-arch=gfx950, one object per translation unit
(compiled in parallel), linked against the HIP runtime and RCCL.  No JIT cache is involved, so
the built .so travels with the repository snapshot to the GPU box."""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.environ.get("DSSM_CSRC_DIR", os.path.join(PKG, "csrc"))  # side builds: a patched copy
# DSSM_BUILD_TAG: a side build (A/B variants of DSSM_EXTRA_CFLAGS) in _build<tag>/, libdssm<tag>.so
TAG = os.environ.get("DSSM_BUILD_TAG", "")
OBJ = os.path.join(PKG, "_build" + TAG)
LIB = os.path.join(PKG, f"libdssm{TAG}.so")
SOURCES = ["spmm.hip", "gemm.hip", "gemm32.hip", "bn.hip", "cosine.hip", "adam.hip", "plan.hip", "feed.hip", "rnn.hip", "rnn_mfma.hip", "ops.hip", "peer.hip"]
HEADERS = ["common.h", "launch.h", "gather.h", "bnfuse.h", "flat.h", "tn.h", "csc.h", "g32.h"]
ARCH = os.environ.get("DSSM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]
CFLAGS += os.environ.get("DSSM_EXTRA_CFLAGS", "").split()  # diagnostics builds (e.g. -DDSSM_WG_TL)


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def _deps_mtime():
    hs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "dssm.h")]
    return max(_mtime(h) for h in hs)


def _compile(src: str, force: bool) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src.replace(".hip", ".o"))
    if not force and _mtime(o) > max(_mtime(s), _deps_mtime()):
        return o
    cmd = [HIPCC, *CFLAGS, "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return o


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[dssm_amd] built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
