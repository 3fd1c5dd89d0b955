"""Generate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference ships no tests, fixtures or golden vectors and its TensorFlow graph cannot run
here (TF absent, no network), so these vectors come from the oracle (oracle/dssm_oracle.py,
float64) on seeded synthetic batches (dssm_amd/data.py) — they pin the GPU path to the oracle
and the oracle to itself across edits; TF-level parity stays unpinned.

Each fixture holds, for one configuration: three training batches (combined CSR), the initial
parameters, step-1 outputs (loss, accuracy, cos_sim_raw, prob, all gradients, batch moments),
the full optimizer state (params, Adam m/v, EMA) after steps 1 and 2, per-step masks of the
well-conditioned gradient elements, the parameters / EMA shadows / losses after three Adam
steps, and an eval-mode (EMA) forward on a fourth batch.  Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import dssm_oracle as O  # noqa: E402
from dssm_amd.data import synth_batch  # noqa: E402

CASES = {
    "tiny": dict(D=64, widths=[16, 16], BS=8, NEG=4, mean_nnz=8, seed=5),
    "c1": dict(D=1000, widths=[100, 100], BS=128, NEG=4, mean_nnz=32, seed=7),
    "c1_3layer": dict(D=500, widths=[100, 100, 64], BS=32, NEG=3, mean_nnz=24, seed=9),
}


def build_case(c):
    cfg = O.OracleConfig(trigram_d=c["D"], widths=list(c["widths"]), query_bs=c["BS"], neg=c["NEG"])
    out = {}
    p = O.init_params(cfg, seed=c["seed"])
    for k, v in p.items():
        out[f"p0__{k}"] = v.copy()
    batches = [synth_batch(c["D"], c["BS"], c["NEG"], seed=1000 * c["seed"] + b,
                           mean_nnz=c["mean_nnz"]) for b in range(4)]
    for b, bt in enumerate(batches):
        out[f"batch{b}__indptr"] = bt.indptr
        out[f"batch{b}__indices"] = bt.indices
        out[f"batch{b}__values"] = bt.values
    ema = O.make_ema(cfg)
    adam = O.AdamState(cfg, p)
    losses = []
    for step in range(3):
        cache, grads, ema = O.train_step(cfg, p, ema, adam, batches[step].as_dict(), dtype=np.float64)
        losses.append(cache["loss"])
        # elements whose gradient is well above the rounding level of its cancelling terms
        for k, g in grads.items():
            out[f"well{step + 1}__{k}"] = np.packbits((np.abs(g) > 1e-3 * np.abs(g).max()).reshape(-1))
        if step < 2:  # full state after steps 1 and 2 for teacher-forced single-step checks
            s = step + 1
            for k in p:
                out[f"p{s}__{k}"] = p[k].copy()
                out[f"m{s}__{k}"] = adam.m[k].copy()
                out[f"v{s}__{k}"] = adam.v[k].copy()
            for k, v in ema.items():
                out[f"ema{s}__{k}"] = v.copy()
        if step == 0:
            out["s1__loss"] = np.float64(cache["loss"])
            out["s1__accuracy"] = np.float64(cache["accuracy"])
            out["s1__cos_sim_raw"] = cache["cos_sim_raw"]
            out["s1__prob"] = cache["prob"]
            for k, g in grads.items():
                out[f"g1__{k}"] = np.asarray(g, np.float64)
            for l, lc in enumerate(cache["layers"], start=1):
                for t in ("q", "d"):
                    out[f"s1__bn{l}_{t}_batch_mean"] = lc["batch_mean"][t]
                    out[f"s1__bn{l}_{t}_batch_var"] = lc["batch_var"][t]
    out["losses"] = np.array(losses)
    for k, v in p.items():
        out[f"p3__{k}"] = v.copy()
    for k, v in ema.items():
        out[f"ema3__{k}"] = v.copy()
    ev = O.forward(cfg, p, ema, batches[3].as_dict(), train=False, dtype=np.float64)[0]
    out["eval__loss"] = np.float64(ev["loss"])
    out["eval__cos_sim_raw"] = ev["cos_sim_raw"]
    return out


def main():
    for name, c in CASES.items():
        d = build_case(c)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB, {len(d)} arrays)")


if __name__ == "__main__":
    main()
