"""Diagnostics (GPU box): build and replay the data-parallel step graph at world 1 with each comm
mode (1 copies, 2 modelled, 0 RCCL), printing progress, to isolate a failure."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dssm_amd import _lib  # noqa: E402
from tests.test_gpu_parity import make  # noqa: E402
from tests.test_gpu_wire import D, WIDTHS, BS, NEG, _staged, _wires  # noqa: E402

modes = [int(x) for x in sys.argv[1:]] or [1, 2, 0]
lib = _lib.load()
for comm in modes:
    if comm == 0 and lib.dssm_comm_world() == 0:
        buf = (C.c_char * 128)()
        _lib.check(lib.dssm_comm_unique_id(buf), "id")
        _lib.check(lib.dssm_comm_init(0, 1, buf), "init")
        print("comm init ok", flush=True)
    _, _, m = make(D, WIDTHS, BS, NEG, "bf16", fused=False)
    _wires(m, 1, 0, 3)
    batches = _staged([300, 301])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        print("building comm", comm, flush=True)
        gid = m.graph_build_dp_steps(batches, 1.0, comm=comm, link_gbps=100.0, latency_us=5.0)
        print("built", flush=True)
        m.graph_launch(gid)
    torch.cuda.synchronize()
    print("comm", comm, "ok loss", m.loss_accuracy(), flush=True)
