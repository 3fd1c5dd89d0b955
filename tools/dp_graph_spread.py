"""Diagnostics: the spread behind tests/test_gpu_wire.py::test_dp_step_graph_default_schedule_matches_eager
(default schedule, fp32 column-sum atomics): for its (comm 0, 1 chunk, BS 128, 2 replays) case, the
fraction of parameters within 1e-4 for graph-vs-eager and for eager-vs-eager, several repetitions.
    python3 tools/dp_graph_spread.py [BS CHUNKS]   (default 128 1)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make
from tests.test_gpu_wire import D, NEG, WIDTHS, _wires


BS_, CHUNKS = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (128, 1)


def run(mode, batches, chunks, replays, comm=0):
    _, _, m = make(D, WIDTHS, BS_, NEG, "bf16", fused=False)
    gw, st, pw, geo = _wires(m, 1, 0, chunks)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        if mode == "graph":
            gid = m.graph_build_dp_steps(batches, 1.0, comm=comm)
            for _ in range(replays):
                m.graph_launch(gid)
        else:
            for _ in range(replays):
                for ip, ix, vv in batches:
                    m.set_batch(indptr=ip, indices=ix, values=vv)
                    m.forward(True)
                    m.backward()
                    st.copy_(gw)
                    m.apply_adam(1.0)
                    m.wire_shadows()
    torch.cuda.synchronize()
    return m.params.clone()


import ctypes as C

from dssm_amd import _lib

lib = _lib.load()
if lib.dssm_comm_world() == 0:  # libdssm.so's RCCL communicator at world 1 (as the test's fixture)
    buf = (C.c_char * 128)()
    _lib.check(lib.dssm_comm_unique_id(buf), "comm_unique_id")
    _lib.check(lib.dssm_comm_init(0, 1, buf), "comm_init")
batches = []
for i in range(3):
    b = synth_batch(D, BS_, NEG, seed=300 + i, mean_nnz=32)
    batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
for rep in range(4):
    g, e1, e2 = run("graph", batches, CHUNKS, 2), run("eager", batches, CHUNKS, 2), run("eager", batches, CHUNKS, 2)
    f = lambda a, b: float(((a - b).abs() <= 1e-4).float().mean())
    print(f"rep {rep}: graph-vs-eager {f(g, e1):.4f}  eager-vs-eager {f(e1, e2):.4f}  graph-vs-eager2 {f(g, e2):.4f}", flush=True)
lib.dssm_comm_destroy()
