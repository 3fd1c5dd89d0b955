"""CPU baseline timing of the DSSM step — TEST/BENCH INFRASTRUCTURE ONLY (bench.py's
cpu_baseline leg).  The reference's own CPU path (TensorFlow 1.x) cannot run here (TF absent,
no network), so the baseline is the port of the same graph: the C/OpenMP restatement in
oracle/dssm_cpu.c when it is built (kind "port", all host threads), else the NumPy oracle in
float32 (kind "port", NumPy/BLAS threads).  The merge of negatives is a permutation in both, so
the reference's O((BS*NEG)^2) concat chain (new_dssm.py:169-179) is NOT charged to the baseline
— it is conservative in the reference's favour."""
from __future__ import annotations

import os
import time

import numpy as np

from . import dssm_oracle as O


def _threads():
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        if os.environ.get(k):
            try:
                return int(os.environ[k])
            except ValueError:
                pass
    return os.cpu_count() or 1


def host_cpus() -> dict:
    """What the host offers the baseline: the threads used, the process's affinity-mask size, the
    machine's CPU count (nproc) and OMP_NUM_THREADS.  On the GPU box OMP_NUM_THREADS is the box's
    CPU share (16 per GPU), set by the harness and left as it is; nproc counts the whole machine."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"threads_used": _threads(), "affinity_cpus": aff, "nproc": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def time_steps(D, widths, BS, NEG, budget_s: float = 15.0, max_steps: int = 100000, use_c: bool = True,
               scaling=None):
    """use_c=False times the NumPy float32 oracle even when the C port is built (SURVEY §8(d)'s
    secondary CPU number).  scaling: thread counts for the C port's rate-vs-threads record."""
    from dssm_amd.data import ZipfColumns, synth_batch  # synthetic batches only (host numpy)
    if use_c:
        try:
            from . import cpu_c
            if cpu_c.available():
                out = cpu_c.time_steps(D, widths, BS, NEG, budget_s=budget_s, max_steps=max_steps,
                                       scaling=scaling)
                out["host"] = host_cpus()
                return out
        except ImportError:
            pass
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    p = O.init_params(cfg, seed=0)
    ema = O.make_ema(cfg)
    adam = O.AdamState(cfg, p)
    cols = ZipfColumns(D)
    batches = [synth_batch(D, BS, NEG, seed=1000 + b, cols=cols).as_dict() for b in range(2)]
    # one untimed warm-up step
    _, ema = O.train_step(cfg, p, ema, adam, batches[0], dtype=np.float32)[0::2]
    steps, t0 = 0, time.perf_counter()
    while steps < max_steps:
        _, _, ema = O.train_step(cfg, p, ema, adam, batches[steps % 2], dtype=np.float32)
        steps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": round(steps * BS * (NEG + 1) / el, 1), "unit": "pairs/s",
            "cores": _threads(), "kind": "port", "host": host_cpus(),
            "sample": f"{steps} full C2 steps (fwd+bwd+dense Adam, BS={BS}) of the NumPy float32 "
                      f"oracle in {el:.1f}s"}


def time_multiview_steps(cfg, params, feeds, budget_s: float = 15.0, max_steps: int = 10000):
    """multi_view_dssm_v3 (BASELINE config 5) on the host: the oracle's forward / backward / Adam
    (oracle/multiview_oracle.py) in float32 with scipy CSR inputs, so FC1 is a sparse product as in
    the reference's tf.sparse_tensor_dense_matmul (archive/multi_view_dssm_v3.py:121-128).
    feeds: [(user_csr, item_csr, view, rot)]; one untimed warm-up step."""
    from . import multiview_oracle as MV
    p = {k: np.array(v, np.float32) for k, v in params.items()}
    adam = MV.Adam(cfg, p)

    def step(i):
        u, it, view, rot = feeds[i % len(feeds)]
        fw = MV.forward(cfg, p, u, it, view, rot, dtype=np.float32, sparse=True)
        adam.step(p, MV.backward(cfg, p, fw))
    step(0)
    steps, t0 = 0, time.perf_counter()
    while steps < max_steps:
        step(1 + steps)
        steps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": round(steps * cfg.bs * (cfg.neg + 1) / el, 1), "unit": "pairs/s",
            "cores": _threads(), "kind": "port", "host": host_cpus(),
            "sample": f"{steps} full config-5 steps (user + active view fwd + bwd + Adam, BS={cfg.bs}) of "
                      f"the NumPy float32 multi-view oracle with scipy CSR inputs in {el:.1f}s"}
