"""Diagnostics: the round-4 segfault inside torch.cuda.graph's capture_end with
the THREE-stream multi-view step (gpurun_out/mv3/tests.log: test_multiview_fused_graph_matches_eager).

The variant is re-created here as a subclass of the product model (the product keeps two streams):
the two towers' CSC transposes (they depend on the batch only) run on a third stream aux2, forked
from the step's stream at the start of forward(), so the item tower's backward on aux does not queue
behind them; the user tower's optimizer launch (on the capture stream) waits on an event recorded on
aux2 after the user transpose, the item tower's (on aux) on one recorded after the item transpose.

Before the capture ends, every stream's capture state is queried (hipStreamGetCaptureInfo_v2:
status, capture id, the number of nodes its next work would depend on) and printed, then the capture
is ended.  Each configuration runs in a child process so a crash is reported, not fatal:
    python tools/mv_capture_probe.py"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STATUS = {0: "none", 1: "active", 2: "invalidated"}


def capture_info(hip, stream) -> str:
    st, cid = C.c_int(), C.c_ulonglong()
    graph, deps, nd = C.c_void_p(), C.c_void_p(), C.c_size_t()
    rc = hip.hipStreamGetCaptureInfo_v2(C.c_void_p(stream.cuda_stream), C.byref(st), C.byref(cid),
                                        C.byref(graph), C.byref(deps), C.byref(nd))
    return f"rc {rc} status {STATUS.get(st.value, st.value)} id {cid.value} deps {nd.value}"


def child(variant: str, dtype: str):
    import numpy as np
    import torch

    from dssm_amd import _lib
    from dssm_amd._lib import stream_ptr
    from dssm_amd.data import ZipfColumns, synth_rows
    from dssm_amd.multiview import MultiViewDSSM
    from oracle import multiview_oracle as M

    class ThreeStream(MultiViewDSSM):
        """The transposes on a third stream aux2, forked from the step's stream (variant
        "fork_main") or from the item tower's stream aux (variant "fork_aux": a stream forked from a
        forked stream by event waits, the round-4 form)."""
        def __init__(self, *a, fork="main", **k):
            super().__init__(*a, **k)
            self.aux2 = torch.cuda.Stream(self.device)
            self.fork = fork

        def forward(self, stream=None):
            main = self._fork(stream)
            s, sa = stream_ptr(main), stream_ptr(self.aux)
            BS = self.bs
            if self.fork == "main":
                self.aux2.wait_stream(main)
            elif self.fork == "aux":
                self.aux2.wait_stream(self.aux)  # aux was forked from main by _fork, no node of its own yet
            else:  # "aux_late": forked from aux after aux captured a kernel node of its own
                self._tower_fwd("i", f"view{self.view}", self.ysrc[BS:], sa)
                self.aux2.wait_stream(self.aux)
            for key in ("u", "i"):
                for t in self.batch[key]:
                    t.record_stream(self.aux2)
            s2 = stream_ptr(self.aux2)
            self._csc("u", "user", s2)
            self._csc_ev = self.aux2.record_event()
            self._csc("i", f"view{self.view}", s2)
            self._csc_ev_i = self.aux2.record_event()
            self._tower_fwd("u", "user", self.ysrc[:BS], s)
            if self.fork != "aux_late":
                self._tower_fwd("i", f"view{self.view}", self.ysrc[BS:], sa)
            main.wait_event(self.aux.record_event())
            _lib.check(self.lib.dssm_cosine_softmax_loss_mapped(
                _lib.ptr(self.ysrc), self.ld2, _lib.ptr(self.map), self.l2, BS, self.neg, self.gamma,
                _lib.ptr(self.cos_raw), _lib.ptr(self.cos_sim), _lib.ptr(self.prob), _lib.ptr(self.qnorm),
                _lib.ptr(self.loss_buf), _lib.ptr(self.dmerged), _lib.ptr(self.cos_ws), s), "cosine")

        def apply_adam(self, stream=None, grad_scale: float = 1.0):
            main = stream if stream is not None else torch.cuda.current_stream(self.device)
            if not self._adam_pending:
                self._fork(main)
            self._adam_pending = False
            towers = ("user", f"view{self.view}")
            main.wait_event(self._csc_ev)
            self.aux.wait_event(self._csc_ev_i)
            self._tower_adam("u", towers[0], stream_ptr(main), grad_scale, 0, False)
            self._tower_adam("i", towers[1], stream_ptr(self.aux), grad_scale, 1, False)
            main.wait_stream(self.aux)
            self._csc_ev = None
            self.global_step += 1

    hip = C.CDLL("libamdhip64.so")
    cfg = M.MvConfig(user_d=3000, view_d=[2000, 2500, 1500], l1=64, l2=32, bs=512, neg=4, lr=0.01)
    p = M.init_params(cfg, 1)
    rot = M.rotations(cfg, 3)
    fork = variant[len("fork_"):]
    m = ThreeStream(cfg.user_d, cfg.view_d, cfg.l1, cfg.l2, cfg.bs, cfg.neg, lr=cfg.lr, rotations=rot,
                    fused_w1_adam=True, dtype=dtype, fork=fork)
    m.load_params(p)
    rng = np.random.Generator(np.random.PCG64(77))
    feeds = []
    for view in (1, 3):
        uu = synth_rows(rng, ZipfColumns(cfg.user_d), cfg.bs, 16.0)
        ii = synth_rows(rng, ZipfColumns(cfg.view_d[view - 1]), cfg.bs, 16.0)
        m.set_batch(uu, ii, view)
        feeds.append((dict(m.batch), view))
    m.train_step()  # eager step: the variant runs
    torch.cuda.synchronize()
    print(f"[{variant} {dtype}] eager step ok, loss {m.loss():.5f}", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        g.capture_begin()
        for i in range(2):
            m.batch, m.view = dict(feeds[i % 2][0]), feeds[i % 2][1]
            m.forward()
            m.backward(join=False)
            m.apply_adam()
        for name, st in (("capture", s), ("aux", m.aux), ("aux2", m.aux2)):
            print(f"[{variant} {dtype}] before capture_end: {name}: {capture_info(hip, st)}", flush=True)
        g.capture_end()
    print(f"[{variant} {dtype}] capture_end returned", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"[{variant} {dtype}] replay ok, loss {m.loss():.5f}", flush=True)


def main():
    if len(sys.argv) > 2:
        return child(sys.argv[1], sys.argv[2])
    for variant in ("fork_main", "fork_aux_late", "fork_aux"):
        for dtype in ("bf16",):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), variant, dtype], capture_output=True,
                               text=True, timeout=240)
            out = [x for x in (r.stdout + r.stderr).splitlines() if "amdgpu.ids" not in x]
            print("\n".join(out[-12:]))
            print(f"[{variant} {dtype}] exit code {r.returncode}" +
                  (" (SIGSEGV)" if r.returncode in (-11, 139) else ""), flush=True)


if __name__ == "__main__":
    main()
