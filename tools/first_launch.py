"""First-launch cost of region graphs (bench.py times the timed region's graph on its first
launch): which first launches are slow -- the first graph of a size, any fresh graph, or only
graphs larger than every one launched before.  Run on the GPU box: python tools/first_launch.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


def build(k):
    return m.graph_build_steps([staged[i % 16] for i in range(k)])


def launch(g, k, tag):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.graph_launch(g)
    torch.cuda.synchronize()
    us = 1e6 * (time.perf_counter() - t0)
    print(f"{tag:34s} K={k:3d}: {us:8.1f} us  ({us / k:6.1f} us/step)", flush=True)


pre_ms = float(os.environ.get("PRE_MS", "0"))
if pre_ms > 0:  # untimed GPU load before the sequence (clock / power-state warm-up)
    x = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < pre_ms / 1e3:
        x = (x @ x).clamp_(-1, 1)
    torch.cuda.synchronize()
    print(f"pre-load {pre_ms} ms done", flush=True)
touch = int(os.environ.get("TOUCH", "0"))
for _ in range(touch):  # untimed reads of the step's state (caches / TLB warm-up)
    for t in (m.params, m.adam_m, m.adam_v, m.grads, m.workspace):
        t.view(torch.uint8).sum(dtype=torch.int64) if t.dtype == torch.uint8 else t.sum()
    torch.cuda.synchronize()
if touch:
    print(f"touched the state {touch}x", flush=True)
idle_ms = float(os.environ.get("IDLE_MS", "0"))
if idle_ms > 0:
    time.sleep(idle_ms / 1e3)
seq = os.environ.get("SEQ", "5,20,20,40,20,80,40")
gs = {}
for i, k in enumerate(int(x) for x in seq.split(",")):
    fresh = os.environ.get("FRESH", "1") == "1" or k not in gs
    if fresh:
        gs[k] = build(k)
    launch(gs[k], k, f"#{i} {'fresh' if fresh else 'relaunch'}")
    launch(gs[k], k, f"#{i} again")
