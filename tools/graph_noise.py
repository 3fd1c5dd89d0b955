"""Diagnostics: run-to-run spread of free-running steps (two eager runs of the same schedule) next to
graph-vs-eager, for test_gpu_graph's bf16 case (D=5000, 300/300/128, BS=96: the unfused statistics
schedule) -- is the graph path's difference beyond what two eager runs already show?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from dssm_amd.data import synth_batch  # noqa: E402
from dssm_amd.model import DSSM  # noqa: E402
from oracle import dssm_oracle as O  # noqa: E402


def run(case, graph, p, hb, det=False):
    D, widths, BS, NEG, dtype = case
    m = DSSM(D, widths, BS, NEG, dtype=dtype, init=False)
    if det:
        m.set_option("DETERMINISTIC", True)
    m.load_params(p)
    dev = torch.device("cuda:0")
    staged = [(torch.from_numpy(x.indptr).to(dev), torch.from_numpy(x.indices).to(dev),
               torch.from_numpy(x.values).to(dev)) for x in hb]
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        if graph:
            m.graph_launch(m.graph_build_steps(staged, stream=s), stream=s)
        else:
            for ip, ix, vv in staged:
                m.set_batch(indptr=ip, indices=ix, values=vv)
                m.train_step(s)
    s.synchronize()
    return m.params.cpu().numpy().copy()


def frac(a, b):
    d = np.abs(a - b)
    return f"within 1e-4: {float((d <= 1e-4).mean()):.4f}, max {d.max():.2e}"


for case in [(5000, (300, 300, 128), 96, 4, "bf16"), (30000, (300, 300, 128), 128, 4, "fp32")]:
    D, widths, BS, NEG, dtype = case
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=11)
    hb = [synth_batch(D, BS, NEG, seed=3000 + i, mean_nnz=32) for i in range(3)]
    e1, e2 = run(case, False, p, hb), run(case, False, p, hb)
    g1, g2 = run(case, True, p, hb), run(case, True, p, hb)
    d1, d2 = run(case, False, p, hb, det=True), run(case, True, p, hb, det=True)
    print(case, "| eager vs eager:", frac(e1, e2), "| graph vs graph:", frac(g1, g2), "| graph vs eager:",
          frac(g1, e1), "| deterministic graph vs eager:", frac(d2, d1), flush=True)
