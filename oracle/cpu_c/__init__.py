"""ctypes wrapper of oracle/cpu_c/dssm_cpu.c. This is TEST/BENCH INFRASTRUCTURE: the C/OpenMP CPU
restatement of the DSSM step, used as the CPU baseline and checked against the
NumPy oracle in tests/test_cpu_c.py. It is never on the product path.

`build()` compiles the library with gcc (`-O3 -march=x86-64-v3 -fopenmp`: AVX2/FMA, which any
EPYC host of the GPU box runs) into oracle/_build/libdssm_cpu.so. The output is git-ignored and
travels to the GPU box with the snapshot. It is rebuilt there if missing.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from typing import Dict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "dssm_cpu.c")
RNN_SRC = os.path.join(HERE, "rnn_cpu.c")  # the RNN tower's step (BASELINE config 4)
OUT_DIR = os.path.join(os.path.dirname(HERE), "_build")
LIB = os.path.join(OUT_DIR, "libdssm_cpu.so")
MAXL = 8


def build(force: bool = False) -> str:
    if (not force and os.path.exists(LIB)
            and os.path.getmtime(LIB) >= max(os.path.getmtime(SRC), os.path.getmtime(RNN_SRC))):
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + f".tmp{os.getpid()}"
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c11",
                    "-D_POSIX_C_SOURCE=200112L", SRC, RNN_SRC, "-o", tmp, "-lm"], check=True)
    os.replace(tmp, LIB)
    return LIB


def available() -> bool:
    try:
        build()
        return True
    except (OSError, subprocess.CalledProcessError):
        return False


class _Cfg(C.Structure):
    _fields_ = [("D", C.c_int), ("L", C.c_int), ("BS", C.c_int), ("NEG", C.c_int),
                ("widths", C.c_int * MAXL), ("lr", C.c_float), ("beta1", C.c_float),
                ("beta2", C.c_float), ("adam_eps", C.c_float), ("bn_eps", C.c_float),
                ("ema_decay", C.c_float), ("gamma", C.c_float)]


class _Params(C.Structure):
    _fields_ = [("W", C.c_void_p * MAXL), ("b", C.c_void_p * MAXL), ("bn_g", C.c_void_p * MAXL),
                ("bn_b", C.c_void_p * MAXL)]


class _RnnCfg(C.Structure):
    _fields_ = [("V", C.c_int), ("E", C.c_int), ("H", C.c_int), ("T", C.c_int), ("BS", C.c_int),
                ("NEG", C.c_int), ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float),
                ("eps", C.c_float), ("gamma", C.c_float)]


class _RnnParams(C.Structure):
    _fields_ = [("emb", C.c_void_p), ("w", C.c_void_p * 4)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        P = C.c_void_p
        _lib.dssm_cpu_ws_create.restype = P
        _lib.dssm_cpu_ws_create.argtypes = [C.POINTER(_Cfg), C.c_int]
        _lib.dssm_cpu_ws_destroy.argtypes = [P, C.POINTER(_Cfg)]
        _lib.dssm_cpu_train_step.restype = C.c_float
        _lib.dssm_cpu_train_step.argtypes = [C.POINTER(_Cfg), C.POINTER(_Params), C.POINTER(_Params),
                                             C.POINTER(_Params), C.POINTER(_Params), P, P, P, P, P, P]
        _lib.dssm_cpu_forward_backward.restype = C.c_float
        _lib.dssm_cpu_forward_backward.argtypes = [C.POINTER(_Cfg), C.POINTER(_Params), C.POINTER(_Params),
                                                   P, P, P, P, P, C.c_int, C.c_int]
        _lib.dssm_cpu_adam.restype = None
        _lib.dssm_cpu_adam.argtypes = [C.POINTER(_Cfg), C.POINTER(_Params), C.POINTER(_Params),
                                       C.POINTER(_Params), C.POINTER(_Params), P, C.c_float]
        _lib.dssm_cpu_set_threads.restype = C.c_int
        _lib.dssm_cpu_set_threads.argtypes = [C.c_int]
        _lib.dssm_cpu_accuracy.restype = C.c_float
        _lib.dssm_cpu_accuracy.argtypes = [P]
        _lib.rnn_cpu_ws_create.restype = P
        _lib.rnn_cpu_ws_create.argtypes = [C.POINTER(_RnnCfg)]
        _lib.rnn_cpu_ws_destroy.argtypes = [P]
        _lib.rnn_cpu_forward_backward.restype = C.c_float
        _lib.rnn_cpu_forward_backward.argtypes = [C.POINTER(_RnnCfg), C.POINTER(_RnnParams),
                                                  C.POINTER(_RnnParams), P, P, P, P, C.c_float]
        _lib.rnn_cpu_train_step.restype = C.c_float
        _lib.rnn_cpu_train_step.argtypes = [C.POINTER(_RnnCfg), C.POINTER(_RnnParams), C.POINTER(_RnnParams),
                                            C.POINTER(_RnnParams), C.POINTER(_RnnParams), P, P, P, P,
                                            C.c_float, P]
        _lib.rnn_cpu_output.restype = P
        _lib.rnn_cpu_output.argtypes = [P]
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


class CpuDSSM:
    """Holds fp32 params / grads / Adam slots / EMA in the oracle's naming (W{l}, b{l},
    bn{l}_{q|d}_{gamma|beta}; bn{l}_{q|d}_{mean|var})."""

    def __init__(self, D, widths, BS, NEG, params: Dict[str, np.ndarray], lr=0.01, beta1=0.9,
                 beta2=0.999, adam_eps=1e-8, bn_eps=1e-3, ema_decay=0.5, gamma=20.0, max_nnz=None,
                 pad_to: int = 1):
        self.lib = _load()
        L = len(widths)
        self.cfg = _Cfg(D, L, BS, NEG, (C.c_int * MAXL)(*widths), lr, beta1, beta2, adam_eps, bn_eps,
                        ema_decay, gamma)
        self.widths, self.D, self.BS, self.NEG = list(widths), D, BS, NEG
        R = BS * (2 + NEG)
        self.max_nnz = int(max_nnz or R * 96)
        dims = [D] + list(widths)
        self.arrays = {}
        self.structs = {}
        # one flat buffer per role (params, grads, Adam m, Adam v) with named views into it, so the
        # gradient is one contiguous arena like the device path's
        shapes = []
        for l in range(1, L + 1):
            shapes += [(f"W{l}", (dims[l - 1], dims[l])), (f"b{l}", (dims[l],)),
                       (f"bn{l}_g", (2, dims[l])), (f"bn{l}_b", (2, dims[l]))]
        total = sum(int(np.prod(s)) for _, s in shapes)
        self.total = total
        self.flat = {}
        for role in ("p", "g", "m", "v"):
            buf = np.zeros(-(-total // pad_to) * pad_to, np.float32)  # zero tail: equal DP shards
            self.flat[role] = buf
            arr, o = {}, 0
            for name, s in shapes:
                k = int(np.prod(s))
                arr[name] = buf[o:o + k].reshape(s)
                o += k
            self.arrays[role] = arr
            s = _Params()
            for l in range(1, L + 1):
                s.W[l - 1] = _p(arr[f"W{l}"])
                s.b[l - 1] = _p(arr[f"b{l}"])
                s.bn_g[l - 1] = _p(arr[f"bn{l}_g"])
                s.bn_b[l - 1] = _p(arr[f"bn{l}_b"])
            self.structs[role] = s
        self.ema = np.zeros(sum(4 * n for n in widths), np.float32)
        self.beta_powers = np.array([beta1, beta2], np.float32)
        self.set_params(params)
        self.ws = self.lib.dssm_cpu_ws_create(C.byref(self.cfg), self.max_nnz)

    def set_params(self, params):
        a = self.arrays["p"]
        for l in range(1, len(self.widths) + 1):
            a[f"W{l}"][...] = params[f"W{l}"]
            a[f"b{l}"][...] = params[f"b{l}"]
            for i, t in enumerate(("q", "d")):
                a[f"bn{l}_g"][i] = params[f"bn{l}_{t}_gamma"]
                a[f"bn{l}_b"][i] = params[f"bn{l}_{t}_beta"]

    def named(self, role: str) -> Dict[str, np.ndarray]:
        a, out = self.arrays[role], {}
        for l in range(1, len(self.widths) + 1):
            out[f"W{l}"], out[f"b{l}"] = a[f"W{l}"], a[f"b{l}"]
            for i, t in enumerate(("q", "d")):
                out[f"bn{l}_{t}_gamma"] = a[f"bn{l}_g"][i]
                out[f"bn{l}_{t}_beta"] = a[f"bn{l}_b"][i]
        return out

    def named_ema(self) -> Dict[str, np.ndarray]:
        out, o = {}, 0
        for l, n in enumerate(self.widths, start=1):
            for t in ("q", "d"):
                out[f"bn{l}_{t}_mean"] = self.ema[o:o + n]
                out[f"bn{l}_{t}_var"] = self.ema[o + n:o + 2 * n]
                o += 2 * n
        return out

    def _batch(self, batch):
        ip = np.ascontiguousarray(batch["indptr"], np.int32)
        ix = np.ascontiguousarray(batch["indices"], np.int32)
        vv = np.ascontiguousarray(batch["values"], np.float32)
        if ix.size > self.max_nnz:
            raise ValueError("batch nnz exceeds max_nnz")
        return ip, ix, vv

    def train_step(self, batch) -> float:
        ip, ix, vv = self._batch(batch)
        s = self.structs
        return float(self.lib.dssm_cpu_train_step(C.byref(self.cfg), C.byref(s["p"]), C.byref(s["g"]),
                                                  C.byref(s["m"]), C.byref(s["v"]), _p(self.ema), self.ws,
                                                  _p(ip), _p(ix), _p(vv), _p(self.beta_powers)))

    def forward_backward(self, batch, train=True, backward=True) -> float:
        ip, ix, vv = self._batch(batch)
        s = self.structs
        return float(self.lib.dssm_cpu_forward_backward(C.byref(self.cfg), C.byref(s["p"]), C.byref(s["g"]),
                                                        _p(self.ema), self.ws, _p(ip), _p(ix), _p(vv),
                                                        1 if train else 0, 1 if backward else 0))

    def adam(self, grad_scale: float = 1.0):
        s = self.structs
        self.lib.dssm_cpu_adam(C.byref(self.cfg), C.byref(s["p"]), C.byref(s["g"]), C.byref(s["m"]),
                               C.byref(s["v"]), _p(self.beta_powers), float(grad_scale))

    def accuracy(self) -> float:
        return float(self.lib.dssm_cpu_accuracy(self.ws))

    def __del__(self):
        try:
            if getattr(self, "ws", None):
                self.lib.dssm_cpu_ws_destroy(self.ws, C.byref(self.cfg))
                self.ws = None
        except Exception:
            pass


def _threads() -> int:
    v = os.environ.get("OMP_NUM_THREADS")
    try:
        return int(v) if v else (os.cpu_count() or 1)
    except ValueError:
        return os.cpu_count() or 1


def time_steps(D, widths, BS, NEG, budget_s: float = 15.0, max_steps: int = 200, scaling=None,
               scaling_budget_s: float = 2.5):
    """Timed full C2 training steps of the C/OpenMP restatement on synthetic batches, on the
    process's OpenMP team (OMP_NUM_THREADS: the box's CPU share).  scaling: thread counts (each at
    most that team) whose rates are also timed, scaling_budget_s each (at least 2 steps), reported
    as "scaling" {threads: pairs/s} -- how the port's rate grows with cores, for reading the
    GPU / CPU ratio against a whole host."""
    from dssm_amd.data import ZipfColumns, synth_batch
    from .. import dssm_oracle as O
    cfg = O.OracleConfig(trigram_d=D, widths=list(widths), query_bs=BS, neg=NEG)
    m = CpuDSSM(D, widths, BS, NEG, O.init_params(cfg, seed=0))
    cols = ZipfColumns(D)
    batches = [synth_batch(D, BS, NEG, seed=1000 + b, cols=cols).as_dict() for b in range(4)]
    team = m.lib.dssm_cpu_set_threads(0)

    def rate(budget, cap, min_steps=1):
        steps, t0 = 0, time.perf_counter()
        while steps < cap:
            m.train_step(batches[steps % len(batches)])
            steps += 1
            if steps >= min_steps and time.perf_counter() - t0 >= budget:
                break
        return steps, time.perf_counter() - t0
    m.train_step(batches[0])  # untimed warm-up
    steps, el = rate(budget_s, max_steps)
    out = {"value": round(steps * BS * (NEG + 1) / el, 1), "unit": "pairs/s", "cores": team,
           "kind": "port",
           "sample": f"{steps} full C2 training steps (fwd+bwd+dense Adam, BS={BS}, NEG={NEG}) of the "
                     f"C/OpenMP fp32 restatement (oracle/cpu_c) in {el:.1f}s on {team} threads"}
    if scaling:
        sc = {}
        for n in sorted({int(x) for x in scaling if 0 < int(x) <= team}):
            m.lib.dssm_cpu_set_threads(n)
            m.train_step(batches[1])  # untimed: the new team's first step
            k, t = rate(scaling_budget_s, max_steps, min_steps=2)
            sc[str(n)] = round(k * BS * (NEG + 1) / t, 1)
        m.lib.dssm_cpu_set_threads(team)
        out["scaling"] = {"threads_to_pairs_per_s": sc,
                          "sample": f"full C2 steps, >= {scaling_budget_s}s (>= 2 steps) per thread count"}
    return out


class CpuRnnDSSM:
    """The RNN tower's step in C (rnn_cpu.c) over the oracle's parameter names (emb, {fw,bw}_{Wg,bg,
    Wc,bc}); the GRU blocks are stored as [W; b] like the GPU arena."""

    BLOCKS = ("fw_g", "fw_c", "bw_g", "bw_c")

    def __init__(self, nwords, emb, hidden, query_bs, neg, seq_len, params, lr=1e-5, beta1=0.9,
                 beta2=0.999, eps=1e-8, gamma=20.0):
        self.lib = _load()
        self.cfg = _RnnCfg(nwords, emb, hidden, seq_len, query_bs, neg, lr, beta1, beta2, eps, gamma)
        self.E, self.H, self.R = emb, hidden, query_bs * (2 + neg)
        K = emb + hidden
        shapes = {"emb": (nwords, emb), "fw_g": (K + 1, 2 * hidden), "fw_c": (K + 1, hidden),
                  "bw_g": (K + 1, 2 * hidden), "bw_c": (K + 1, hidden)}
        self.arrays, self.structs = {}, {}
        for role in ("p", "g", "m", "v"):
            arr = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
            st = _RnnParams()
            st.emb = _p(arr["emb"])
            for i, k in enumerate(self.BLOCKS):
                st.w[i] = _p(arr[k])
            self.arrays[role], self.structs[role] = arr, st
        self.set_params(params)
        self.beta_powers = np.array([beta1, beta2], np.float32)
        self.ws = self.lib.rnn_cpu_ws_create(C.byref(self.cfg))

    def set_params(self, p):
        a = self.arrays["p"]
        a["emb"][...] = p["emb"]
        for d in ("fw", "bw"):
            a[f"{d}_g"][...] = np.concatenate([p[f"{d}_Wg"], p[f"{d}_bg"][None, :]], 0)
            a[f"{d}_c"][...] = np.concatenate([p[f"{d}_Wc"], p[f"{d}_bc"][None, :]], 0)

    def named(self, role: str) -> Dict[str, np.ndarray]:
        a = self.arrays[role]
        K = self.E + self.H
        out = {"emb": a["emb"]}
        for d in ("fw", "bw"):
            out[f"{d}_Wg"], out[f"{d}_bg"] = a[f"{d}_g"][:K], a[f"{d}_g"][K]
            out[f"{d}_Wc"], out[f"{d}_bc"] = a[f"{d}_c"][:K], a[f"{d}_c"][K]
        return out

    def _args(self, ids, lens, mask):
        ids = np.ascontiguousarray(ids, np.int32)
        lens = np.ascontiguousarray(lens, np.int32)
        m = None if mask is None else np.ascontiguousarray(mask, np.float32)
        return ids, lens, m

    def forward_backward(self, ids, lens, mask=None, keep=1.0, backward=True) -> float:
        ids, lens, m = self._args(ids, lens, mask)
        s = self.structs
        return float(self.lib.rnn_cpu_forward_backward(C.byref(self.cfg), C.byref(s["p"]),
                                                       C.byref(s["g"]) if backward else None, self.ws,
                                                       _p(ids), _p(lens), None if m is None else _p(m),
                                                       float(keep)))

    def train_step(self, ids, lens, mask=None, keep=1.0) -> float:
        ids, lens, m = self._args(ids, lens, mask)
        s = self.structs
        return float(self.lib.rnn_cpu_train_step(C.byref(self.cfg), C.byref(s["p"]), C.byref(s["g"]),
                                                 C.byref(s["m"]), C.byref(s["v"]), self.ws, _p(ids), _p(lens),
                                                 None if m is None else _p(m), float(keep),
                                                 _p(self.beta_powers)))

    def output(self) -> np.ndarray:
        ptr = self.lib.rnn_cpu_output(self.ws)
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_float)), shape=(self.R, 2 * self.H)).copy()

    def __del__(self):
        try:
            if getattr(self, "ws", None):
                self.lib.rnn_cpu_ws_destroy(self.ws)
                self.ws = None
        except Exception:
            pass


def rnn_time_steps(nwords, emb, hidden, query_bs, neg, seq_len, params, batches, keep=0.5,
                   budget_s: float = 15.0):
    """Bounded timing of full RNN-tower steps (fwd + BPTT + Adam) on all host threads."""
    from .. import rnn_oracle as RO
    m = CpuRnnDSSM(nwords, emb, hidden, query_bs, neg, seq_len, params)
    R = query_bs * (2 + neg)
    lens = np.full(R, seq_len, np.int32)
    masks = [RO.dropout_mask(R, 2 * hidden, keep, 0, i + 1) for i in range(2)]
    m.train_step(batches[0], lens, masks[0], keep)  # untimed warm-up (page faults, thread pool)
    n, t0 = 0, time.perf_counter()
    while n < 1 or time.perf_counter() - t0 < budget_s:
        m.train_step(batches[n % len(batches)], lens, masks[n % 2], keep)
        n += 1
    el = time.perf_counter() - t0
    return {"value": round(query_bs * (neg + 1) * n / el, 1), "unit": "pairs/s", "cores": _threads(),
            "kind": "port",
            "sample": f"{n} full config-4 steps (fwd + BPTT + Adam, BS={query_bs}, T={seq_len}) of the "
                      f"C/OpenMP fp32 restatement (oracle/cpu_c/rnn_cpu.c) in {el:.1f}s"}
