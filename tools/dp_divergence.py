"""Diagnostics: WHERE two eager runs of the default (non-deterministic) data-parallel step part ways
(the bimodal spread of tests/test_gpu_wire.py::test_dp_step_graph_default_schedule_matches_eager's
BS-128 one-chunk case, profiles/r05_dp_graph_spread.txt).

NRUNS eager runs of the same 6 steps (3 batches x 2) from the same state on the world-1 bf16 wire
(the test's shapes), every intermediate snapshotted per step: the layers' Z (fp32 pre-BN), the
ReLU masks of A, dZ (bf16), cos_sim_raw, loss, W1's bf16 gradient wire, the fp32 gradient arena
(tail), and after Adam params / m / v.  Each run is compared with run 0 per step and tensor:
elements differing at all, max |diff|, ReLU mask flips, and for the parameters the elements now
more than 1e-4 apart with the gradient each run fed Adam there (sign flips, |g| relative to the
tensor's max).
With V > 0 every run starts from a mid-training Adam state (v = V everywhere, m = 0, beta powers at
step 100) instead of the fresh one.  A graph run (the test's captured 3-step DP graph, two replays,
RCCL at world 1) is compared with the eager runs as well, by parameters (absolute) and by the
update each run applied (p_end - p_start, relative to the eager run's update).
    python3 tools/dp_divergence.py [NRUNS BS CHUNKS V]   (default 4 128 1 0)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dssm_amd import _lib
from dssm_amd.data import synth_batch
from tests.test_gpu_parity import make
from tests.test_gpu_wire import D, NEG, WIDTHS, _wires

NRUNS, BS_, CHUNKS = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (4, 128, 1)
VWARM = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
WARM = VWARM > 0


def warm_state(m):
    """A mid-training Adam state: v = VWARM for every element, m = 0, beta powers at step 100."""
    m.adam_v.fill_(VWARM)
    m.adam_m.zero_()
    m.set_beta_powers(0.9 ** 100, 0.999 ** 100)


L = len(WIDTHS)


def snap(m, gw):
    t = {}
    for l in range(L):
        ld = (WIDTHS[l] + 7) // 8 * 8
        t[f"Z{l + 1}"] = m.buffer(_lib.BUF_Z, l).view(m.rows, ld)[:, :WIDTHS[l]].clone()
        a = m.buffer(_lib.BUF_A, l, dtype=torch.bfloat16 if l < L - 1 else torch.float32)
        t[f"mask{l + 1}"] = (a.view(m.rows, ld)[:, :WIDTHS[l]].float() > 0)
    return t


def snap_bwd(m, gw):
    t = {}
    for l in range(L):
        ld = (WIDTHS[l] + 7) // 8 * 8
        t[f"dZ{l + 1}"] = m.buffer(_lib.BUF_DZ, l, dtype=torch.bfloat16).view(m.rows, ld)[:, :WIDTHS[l]].float().clone()
    t["gW1"] = gw[:D * WIDTHS[0]].float().clone()
    ext = m.wire_extent()
    t["g_tail"] = m.grads[ext:m.n_params].clone()
    t["g_arena"] = m.grads.clone()
    return t


def run_graph(batches):
    _, _, m = make(D, WIDTHS, BS_, NEG, "bf16", fused=False)
    if WARM:
        warm_state(m)
    _wires(m, 1, 0, CHUNKS)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        gid = m.graph_build_dp_steps(batches, 1.0, comm=0)
        for _ in range(2):
            m.graph_launch(gid)
    torch.cuda.synchronize()
    return m.params[:m.n_params].clone()


def run(batches):
    _, _, m = make(D, WIDTHS, BS_, NEG, "bf16", fused=False)
    if WARM:
        warm_state(m)
    gw, st, pw, geo = _wires(m, 1, 0, CHUNKS)
    out = []
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for rep in range(2):
            for ip, ix, vv in batches:
                m.set_batch(indptr=ip, indices=ix, values=vv)
                m.forward(True)
                torch.cuda.synchronize()
                rec = snap(m, gw)
                rec["cos"] = torch.from_numpy(m.fetch("cos_sim_raw").ravel().copy())
                m.backward()
                st.copy_(gw)
                torch.cuda.synchronize()
                rec.update(snap_bwd(m, gw))
                m.apply_adam(1.0)
                m.wire_shadows()
                torch.cuda.synchronize()
                rec["params"] = m.params[:m.n_params].clone()
                rec["adam_m"] = m.adam_m[:m.n_params].clone()
                rec["loss"] = m.loss_accuracy()[0]
                out.append(rec)
    return out, m


def by_name(m, diff_arena):
    """Elements differing per named tensor (W1 .. bn*_beta) of a full-arena difference."""
    full = torch.zeros(m.params.numel(), device=diff_arena.device)
    full[:diff_arena.numel()] = diff_arena
    return {k: int((v != 0).sum()) for k, v in m._named_views(full).items() if int((v != 0).sum())}


def main():
    batches = []
    for i in range(3):
        b = synth_batch(D, BS_, NEG, seed=300 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    import ctypes as C
    lib = _lib.load()
    if lib.dssm_comm_world() == 0:  # libdssm.so's RCCL communicator at world 1 (the graph run)
        buf = (C.c_char * 128)()
        _lib.check(lib.dssm_comm_unique_id(buf), "comm_unique_id")
        _lib.check(lib.dssm_comm_init(0, 1, buf), "comm_init")
    runs = []
    for r in range(NRUNS):
        recs, m = run(batches)
        runs.append(recs)
    _, _, m0 = make(D, WIDTHS, BS_, NEG, "bf16", fused=False)
    p0 = m0.params[:m0.n_params].clone()

    def upd_frac(pa, pb, rel):
        """Fraction of elements whose update (p - p0) agrees within rel x |eager update| + rel x
        max |eager update| (the floor covers elements the step barely moves)."""
        ua, ub = pa - p0, pb - p0
        return float(((ua - ub).abs() <= rel * ub.abs() + rel * float(ub.abs().max())).float().mean())
    print(f"# tools/dp_divergence.py: {NRUNS} eager runs, D {D}, widths {WIDTHS}, BS {BS_}, chunks {CHUNKS}, "
          f"default schedule, {f'warm (v = {VWARM:g}, step 100)' if WARM else 'fresh'} Adam state; each run against run 0",
          flush=True)
    fr = lambda a, b, t: float(((a - b).abs() <= t).float().mean())  # noqa: E731
    for tol in (1e-4, 1e-5, 1e-6):
        final = [fr(runs[r][-1]["params"], runs[0][-1]["params"], tol) for r in range(NRUNS)]
        print(f"# final fraction of params within {tol:g} of run 0: " + " ".join(f"{f:.6f}" for f in final))
    gp = run_graph(batches)
    for tol in (1e-4, 1e-5, 1e-6):
        print(f"# graph (2 replays of the 3-step DP graph) within {tol:g} of eager runs: "
              + " ".join(f"{fr(gp, runs[r][-1]['params'], tol):.6f}" for r in range(NRUNS)))
    for rel in (1e-2, 1e-3, 1e-4):
        print(f"# update (p - p0) within {rel:g} relative of run 0's: eager runs "
              + " ".join(f"{upd_frac(runs[r][-1]['params'], runs[0][-1]['params'], rel):.6f}" for r in range(NRUNS))
              + f"; graph {upd_frac(gp, runs[0][-1]['params'], rel):.6f}")
    first = runs[0][0]
    for r in range(1, NRUNS):
        for i in range(len(runs[0])):
            a, b = runs[0][i], runs[r][i]
            dg = by_name(m, (a["g_arena"] - b["g_arena"])[:m.n_params])
            dp = by_name(m, a["params"] - b["params"])
            if dg or dp:
                print(f"# run {r}: first differing step {i}: gradient elements by tensor {dg}; "
                      f"parameter elements by tensor {dp}")
                break
    del first
    for r in range(1, NRUNS):
        print(f"## run {r} vs run 0 (final within 1e-4: {fr(runs[r][-1]['params'], runs[0][-1]['params'], 1e-4):.4f})")
        for i in range(len(runs[0])):
            a, b = runs[0][i], runs[r][i]
            parts = [f"step {i}: loss {a['loss']:.6f}/{b['loss']:.6f}"]
            for k in a:
                if k in ("loss",):
                    continue
                x, y = a[k], b[k]
                if x.dtype == torch.bool:
                    nf = int((x != y).sum())
                    if nf:
                        parts.append(f"{k} flips {nf}")
                    continue
                d = (x.float() - y.float()).abs()
                nd = int((d > 0).sum())
                if nd == 0:
                    continue
                sc = float(x.float().abs().max())
                s = f"{k} ndiff {nd} max {float(d.max()):.2e} (rel {float(d.max()) / max(sc, 1e-30):.1e})"
                if k == "params":
                    far = d > 1e-4
                    nfar = int(far.sum())
                    s += f" >1e-4: {nfar}"
                    if nfar:
                        # the gradient each run fed Adam there (W1 elements: the bf16 wire)
                        idx = far.nonzero().flatten()
                        idx = idx[idx < D * WIDTHS[0]]
                        if idx.numel():
                            ga, gb = a["gW1"][idx], b["gW1"][idx]
                            gmax = float(a["gW1"].abs().max())
                            flip = float(((ga > 0) != (gb > 0)).float().mean())
                            rows = torch.unique(idx // WIDTHS[0])
                            s += (f" [W1: {idx.numel()} in {rows.numel()} rows; grad sign differs {flip:.2f}; "
                                  f"median |g|/max {float(ga.abs().median()) / max(gmax, 1e-30):.1e}]")
                parts.append(s)
            print("  " + "; ".join(parts), flush=True)


if __name__ == "__main__":
    main()
