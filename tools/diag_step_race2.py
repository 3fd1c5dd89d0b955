"""Diagnostics: the 4-step eager sequence of test_cycle_graph_with_rank_in_adam repeated from the
same initial state; per step, report runs whose parameters differ from run 0."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_parity import make
from tests.test_gpu_graph import _batches

D, widths, BS, NEG = 5000, (300, 300, 128), 128, 4
NREP = int(sys.argv[1]) if len(sys.argv) > 1 else 30
batches = _batches(D, BS, NEG, 4)
refs = None
s = torch.cuda.Stream()
for rep in range(NREP):
    _, _, m = make(D, widths, BS, NEG, "bf16")
    torch.cuda.synchronize()
    snaps = []
    with torch.cuda.stream(s):
        for hb in batches:
            m.set_batch(hb)
            m.train_step()
            torch.cuda.synchronize()
            snaps.append((m.params.clone(), m.adam_v.clone(), m.ema.clone(), m.loss_accuracy()[0]))
    if refs is None:
        refs = snaps
        continue
    for i, ((p, v, e, l), (rp, rv, re_, rl)) in enumerate(zip(snaps, refs)):
        d = (p - rp).abs()
        if float(d.max()) > 1e-5 or l != rl:
            n1 = widths[0]
            bad = torch.nonzero(d > 1e-5).flatten().cpu().numpy()
            w1 = bad[bad < (D + 1) * n1]
            rows = np.unique(w1 // n1)
            cnt = np.bincount(batches[i].indices, minlength=D)
            de = (e - re_).abs()
            print(f"rep {rep} step {i}: loss {l:.6f} vs {rl:.6f}; {bad.size} params > 1e-5 (max {float(d.max()):.3e}); "
                  f"ema max diff {float(de.max()):.3e}; W1 rows {rows[:12]} entries {[int(cnt[r]) if r < D else -1 for r in rows[:12]]}; "
                  f"non-W1 {bad[bad >= (D + 1) * n1][:8]}", flush=True)
            break
print("done", NREP, flush=True)
