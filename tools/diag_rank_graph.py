"""Diagnostics: multi-step graph (merged CSC, RANK_IN_ADAM on / off) vs eager steps, teacher-forced
per step (tests/test_gpu_graph.py::test_cycle_graph_with_rank_in_adam)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_parity import make
from tests.test_gpu_graph import _batches, _copy_state
from dssm_amd.data import synth_batch

D, widths, BS, NEG, lr, k = 5000, (300, 300, 128), 128, 4, 0.01, 4
import sys as _s
NT = int(_s.argv[1]) if len(_s.argv) > 1 else 2
for hosted in (False, True):
    for trial in range(NT):
        _, _, ea = make(D, widths, BS, NEG, "bf16")
        _, _, gr = make(D, widths, BS, NEG, "bf16")
        gr.set_option("RANK_IN_ADAM", hosted)
        batches = [synth_batch(D, BS, NEG, seed=2000 + i, mean_nnz=32, uniform=True) for i in range(k)] if os.environ.get('UNIFORM') else _batches(D, BS, NEG, k)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            staged = [tuple(torch.from_numpy(x).cuda() for x in (hb.indptr, hb.indices, hb.values)) for hb in batches]
            gid = gr.graph_build_steps(staged)
            out = []
            for ip, ix, vv in staged:
                ea.set_batch(indptr=ip, indices=ix, values=vv)
                ea.train_step()
                torch.cuda.synchronize()
                out.append(ea.loss_accuracy()[0])
            gr.graph_launch(gid)
            torch.cuda.synchronize()
            d = (ea.params - gr.params).abs()
            # a second eager model from the same start: eager-vs-eager noise
            _, _, eb = make(D, widths, BS, NEG, "bf16")
            for ip, ix, vv in staged:
                eb.set_batch(indptr=ip, indices=ix, values=vv)
                eb.train_step()
            torch.cuda.synchronize()
            d2 = (ea.params - eb.params).abs()
        print(f"hosted={hosted} trial={trial} loss eager {out[-1]:.6f} graph {gr.loss_accuracy()[0]:.6f} "
              f"eager2 {eb.loss_accuracy()[0]:.6f} | graph-vs-eager frac<=1e-4 {float((d <= 1e-4).float().mean()):.4f} "
              f"max {float(d.max()):.3e} | eager-vs-eager frac<=1e-4 {float((d2 <= 1e-4).float().mean()):.4f} "
              f"max {float(d2.max()):.3e}", flush=True)
