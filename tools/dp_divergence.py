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
    python3 tools/dp_divergence.py [NRUNS BS CHUNKS]   (default 4 128 1)"""
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
    return t


def run(batches):
    _, _, m = make(D, WIDTHS, BS_, NEG, "bf16", fused=False)
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
    return out, m.wire_extent()


def main():
    batches = []
    for i in range(3):
        b = synth_batch(D, BS_, NEG, seed=300 + i, mean_nnz=32)
        batches.append(tuple(torch.from_numpy(x).cuda() for x in (b.indptr, b.indices, b.values)))
    runs = []
    for r in range(NRUNS):
        recs, ext = run(batches)
        runs.append(recs)
    print(f"# tools/dp_divergence.py: {NRUNS} eager runs, D {D}, widths {WIDTHS}, BS {BS_}, chunks {CHUNKS}, "
          f"default schedule; each run against run 0", flush=True)
    final = [float(((runs[r][-1]["params"] - runs[0][-1]["params"]).abs() <= 1e-4).float().mean())
             for r in range(NRUNS)]
    print("# final fraction of params within 1e-4 of run 0: " + " ".join(f"{f:.4f}" for f in final))
    for r in range(1, NRUNS):
        print(f"## run {r} vs run 0 (final {final[r]:.4f})")
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
