"""Diagnostics: one eager train step repeated from an identical state; report parameters that
differ from the first run (which segment, which W1 rows, their CSC entry counts)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_parity import make
from tests.test_gpu_graph import _batches

D, widths, BS, NEG = 5000, (300, 300, 128), int(sys.argv[1]) if len(sys.argv) > 1 else 128, 4
NREP = int(sys.argv[2]) if len(sys.argv) > 2 else 40
_, _, m = make(D, widths, BS, NEG, "bf16")
batches = _batches(D, BS, NEG, 4)
segs = m.lib and None
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    # advance a few steps so the state is generic
    for hb in batches[:3]:
        m.set_batch(hb)
        m.train_step()
    torch.cuda.synchronize()
    st = {k: getattr(m, k).clone() for k in ("params", "grads", "adam_m", "adam_v", "ema")}
    bp = m.beta_powers()
    hb = batches[3]
    cnt = np.bincount(hb.indices, minlength=D)
    ref = None
    for rep in range(NREP):
        for k, v in st.items():
            getattr(m, k).copy_(v)
        m.set_beta_powers(*bp)
        m.lib.dssm_plan_sync_shadows(m._plan, torch.cuda.current_stream().cuda_stream)
        m.set_batch(hb)
        m.train_step()
        torch.cuda.synchronize()
        p = m.params.clone()
        if ref is None:
            ref = p
            continue
        d = (p - ref).abs()
        bad = torch.nonzero(d > 1e-6).flatten().cpu().numpy()
        if bad.size:
            n1 = widths[0]
            w1 = bad[bad < (D + 1) * n1]
            rows = np.unique(w1 // n1)
            print(f"rep {rep}: {bad.size} params differ (max {float(d.max()):.3e}); W1 rows {rows[:20]} "
                  f"entries {[int(cnt[r]) if r < D else -1 for r in rows[:20]]}; non-W1 {bad[bad >= (D + 1) * n1][:10]}",
                  flush=True)
    print("done", NREP, flush=True)
