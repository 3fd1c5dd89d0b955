#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
python3 - <<'PY'
import numpy as np
from dssm_amd.data import synth_batch
b = synth_batch(30000, 1024, 4, seed=1000)
with open("gpurun_out/csr.bin", "wb") as f:
    np.array([b.indptr.size - 1, b.indices.size, 30000], np.int32).tofile(f)
    b.indptr.astype(np.int32).tofile(f); b.indices.astype(np.int32).tofile(f); b.values.astype(np.float32).tofile(f)
PY
timeout -k 10 120 tools/ssb gpurun_out/csr.bin
