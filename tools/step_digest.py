"""Digest of the parameters after a few DETERMINISTIC training steps at C2 (both dtypes): run it
once per library build (DSSM_LIB_PATH) to check that a change meant to be bit-exact is.
    DSSM_LIB_PATH=... python3 tools/step_digest.py"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
for dtype in ("bf16", "fp32"):
    m = DSSM(D, W, BS, NEG, dtype=dtype)
    m.init_params(7)
    m.set_option("DETERMINISTIC", True)
    for i in range(3):
        m.set_batch(synth_batch(D, BS, NEG, seed=500 + i, cols=ZipfColumns(D)))
        m.train_step()
    torch.cuda.synchronize()
    h = hashlib.sha256(m.params.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{dtype} loss {m.loss_accuracy()[0]!r} params {h}", flush=True)
