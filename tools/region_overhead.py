"""Where the timed region's fixed cost sits: the bench's single-GPU region graph (K whole steps,
dssm_plan_graph_build_steps) timed three ways for several K -- host wall time around launch +
synchronize (as bench.py), HIP events recorded on the stream just before / after the graph launch
(GPU-side span, includes any idle gap before the first kernel), and the host submission time alone.
Fits time = a + b K for each.  Run on the GPU box: python tools/region_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dssm_amd.data import ZipfColumns, synth_batch
from dssm_amd.model import DSSM

D, W, BS, NEG = 30000, (300, 300, 128), 1024, 4
dev = torch.device("cuda", 0)
m = DSSM(D, W, BS, NEG, dtype="bf16", seed=0, device=dev)
cols = ZipfColumns(D)
staged = []
for b in range(16):
    hb = synth_batch(D, BS, NEG, seed=1000 + b, cols=cols)
    staged.append(tuple(torch.from_numpy(x).to(dev) for x in (hb.indptr, hb.indices, hb.values)))
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
Ks = [1, 2, 5, 10, 20, 40, 100, 200]
graphs = {k: m.graph_build_steps([staged[i % 16] for i in range(k)]) for k in Ks}
warm = m.graph_build_steps([staged[i % 16] for i in range(5)])
def timed(g):
    m.graph_launch(warm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    m.graph_launch(g)
    e1.record(s)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0), 1e3 * e0.elapsed_time(e1), 1e6 * th

# the FIRST launch of a freshly built K = 20 graph against its later launches (bench.py times the
# region graph's first launch)
for trial in range(2):
    g20 = m.graph_build_steps([staged[i % 16] for i in range(20)])
    first = timed(g20)
    later = [timed(g20) for _ in range(3)]
    print(f"K=20 fresh graph: first launch wall {first[0]:.1f} event {first[1]:.1f} submit {first[2]:.1f} us; "
          f"later {[round(x[0], 1) for x in later]}")
rows = []
for rep in range(3):
    for k in Ks:
        m.graph_launch(warm)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(s)
        m.graph_launch(graphs[k])
        e1.record(s)
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        rows.append((k, 1e6 * tw, 1e3 * e0.elapsed_time(e1), 1e6 * th))
rows = np.array(rows)
print(f"{'K':>4} {'wall us':>10} {'event us':>10} {'host submit us':>15}")
for k in Ks:
    r = rows[rows[:, 0] == k]
    med = np.median(r[:, 1:], axis=0)
    print(f"{k:4d} {med[0]:10.1f} {med[1]:10.1f} {med[2]:15.1f}   wall/K {med[0] / k:7.1f}  event/K {med[1] / k:7.1f}")
for j, name in ((1, "wall"), (2, "event"), (3, "host submit")):
    kk = rows[:, 0]
    b, a = np.polyfit(kk, rows[:, j], 1)
    print(f"fit {name}: {a:.1f} us + {b:.2f} us/step")
