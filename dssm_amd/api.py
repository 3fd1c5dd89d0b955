"""The reference's Python API on the MI355X path, so its training loop drops in.

The reference (semantic_matching/dssm/new_dssm.py) builds a TF1.x graph. It uses sparse placeholders
(:111-115), FC/BN name scopes (:117-158), and Merge/Cosine/Loss (:160-213). It drives the graph with
`sess.run(fetch, feed_dict=pull_batch(...))` (:267-328) and exports embeddings by tensor name
(load_model_and_save_vector.py:30-46). This module keeps those names and that feed/fetch contract.

Two halves:

* **Session API.** `DSSMGraph` holds the placeholders and fetch handles named like the reference's
  tensors. `Session.run(fetches, feed_dict)` runs them on the libdssm.so plan. `Saver` saves and
  restores checkpoints. A loop shaped like new_dssm.py:256-331 runs unchanged given
  `dssm_amd.data.pull_batch`.
* **Functional API.** These are forward-only device ops for inference/export:
  * `sparse_tensor_dense_matmul` (FC1, :124-126);
  * `add_layer` (README.md:66-76 / archive dssm_v3);
  * `batch_normalization` (:62-88), with the ReLU fused;
  * `cosine_similarity` (Merge + Cosine_Similarity + Loss, :160-213).

  Each wraps one C-ABI kernel (include/dssm.h). Torch tensors are only device storage.

Everything runs on the GPU through libdssm.so. There is no CPU fallback: a missing library raises
at import of the model (dssm_amd._lib.load).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from types import SimpleNamespace
from typing import Any, Dict, Iterable, Optional

import numpy as np
import torch

from . import _lib, tfckpt
from .data import SparseTensorValue, feeds_to_csr
from .metrics import StreamingAUC, dssm_labels
from .model import DSSM

GAMMA = 20.0  # cos_sim scale (new_dssm.py:199)


# ---- placeholders and fetch handles --------------------------------------------------------
class Placeholder:
    """tf.sparse_placeholder / tf.placeholder stand-in: a hashable feed key with the reference's
    tensor name.  A sparse placeholder also exposes its components (indices/values/shape) the way
    load_model_and_save_vector.py:36-46 feeds them."""

    def __init__(self, name: str, sparse: bool, dense_width: Optional[int] = None):
        self.name = name
        self.sparse = sparse
        self.dense_width = dense_width
        if sparse:
            self.indices = _Component(self, "indices")
            self.values = _Component(self, "values")
            self.shape = _Component(self, "shape")

    def __repr__(self):
        return f"<Placeholder {self.name}>"


class _Component:
    def __init__(self, parent: Placeholder, part: str):
        self.parent, self.part = parent, part
        self.name = f"{parent.name}/{part}"

    def __repr__(self):
        return f"<Placeholder {self.name}>"


def sparse_placeholder(dtype=None, shape=None, name: str = "sparse") -> Placeholder:
    return Placeholder(name, True, None if shape is None else shape[-1])


def placeholder(dtype=None, shape=None, name: str = "placeholder") -> Placeholder:
    return Placeholder(name, False)


class Fetch:
    """A fetchable value of the DSSM graph (reference tensor / op name)."""

    def __init__(self, key: str, name: str):
        self.key, self.name = key, name

    def __repr__(self):
        return f"<Fetch {self.name}>"


# key -> reference name (name scope / tensor), new_dssm.py and load_model_and_save_vector.py
_FETCHES = {
    "train_step": "Training/train_step",
    "loss": "Loss/loss",
    "accuracy": "Accuracy/accuracy",
    "prob": "Loss/prob",
    "cos_sim": "Cosine_Similarity/cos_sim",
    "cos_sim_raw": "Cosine_Similarity/cos_sim_raw",
    "query_norm_single": "Cosine_Similarity/query_norm_single",
    "embedding_query_y": "BN2/embedding_query_y",
    "embedding_doc_positive_y": "BN2/embedding_doc_positive_y",
    "embedding_doc_negative_y": "BN2/embedding_doc_negative_y",
    "auc_op": "Auc/auc_op",
    "auc_value": "Auc/auc_value",
}
_NEEDS_FORWARD = set(_FETCHES) - {"auc_value"}


class DSSMGraph:
    """What new_dssm.py:104-231 builds, bound to one device model.

    conf: dssm_amd.config.Config (reference attribute names: query_BS, L1_N, L2_N, NEG,
    learning_rate; plus L3_N / compute_dtype / max_nnz_per_row)."""

    def __init__(self, conf, trigram_d: int, device=None, seed: Optional[int] = None):
        self.conf = conf
        self.trigram_d = int(trigram_d)
        self.query_BS, self.NEG = int(conf.query_BS), int(conf.NEG)
        self.query_batch = sparse_placeholder(shape=[None, trigram_d], name="input/query_batch")
        self.doc_positive_batch = sparse_placeholder(shape=[None, trigram_d], name="input/doc_positive_batch")
        self.doc_negative_batch = sparse_placeholder(shape=[None, trigram_d], name="input/doc_negative_batch")
        self.on_train = placeholder(name="input/on_train")
        for key, name in _FETCHES.items():
            setattr(self, key, Fetch(key, name))
        # the reference's Python names for the embeddings (new_dssm.py:156-158)
        self.query_y = self.embedding_query_y
        self.doc_positive_y = self.embedding_doc_positive_y
        self.doc_negative_y = self.embedding_doc_negative_y
        rows = self.query_BS * (2 + self.NEG)
        self.model = DSSM(self.trigram_d, conf.widths, self.query_BS, self.NEG, lr=conf.learning_rate,
                          dtype=conf.compute_dtype, max_nnz=rows * int(conf.max_nnz_per_row),
                          device=device, seed=conf.seed if seed is None else seed)
        self.auc = StreamingAUC(2000)
        self._by_name = {self.on_train.name: self.on_train}
        for ph in (self.query_batch, self.doc_positive_batch, self.doc_negative_batch):
            self._by_name[ph.name] = ph
            for comp in (ph.indices, ph.values, ph.shape):
                self._by_name[comp.name] = comp
        for key, name in _FETCHES.items():
            self._by_name[name] = getattr(self, key)
        global _DEFAULT_GRAPH
        _DEFAULT_GRAPH = self

    def meta(self) -> Dict[str, Any]:
        """What import_meta_graph needs to rebuild this graph (written beside a checkpoint as
        <prefix>.meta by Saver.save)."""
        c = self.conf
        return {"format": META_FORMAT, "trigram_d": self.trigram_d, "query_BS": self.query_BS, "NEG": self.NEG,
                "L1_N": c.L1_N, "L2_N": c.L2_N, "L3_N": c.L3_N, "learning_rate": c.learning_rate,
                "compute_dtype": c.compute_dtype, "max_nnz_per_row": c.max_nnz_per_row, "seed": c.seed,
                "tensors": sorted(self._by_name)}

    def get_tensor_by_name(self, name: str):
        """graph.get_tensor_by_name (load_model_and_save_vector.py:30-46); ':0' suffix optional."""
        base = name[:-2] if name.endswith(":0") else name
        if base not in self._by_name:
            raise KeyError(f"no tensor named {name!r} in the DSSM graph")
        return self._by_name[base]


class Session:
    """sess.run over a DSSMGraph: one device forward per run (train- or eval-mode BN per the
    on_train feed), + backward + Adam when train_step is fetched."""

    def __init__(self, graph: Optional[DSSMGraph] = None, stream=None):
        """graph: None = the default graph (the last one built or imported), as tf.Session()."""
        self.graph = graph if graph is not None else get_default_graph()
        self.stream = stream

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def close(self):
        pass

    def _assemble_feeds(self, feed_dict: Dict[Any, Any]):
        g = self.graph
        sparse: Dict[Placeholder, Any] = {}
        parts: Dict[Placeholder, Dict[str, Any]] = {}
        on_train = None
        for k, v in feed_dict.items():
            if isinstance(k, str):
                k = g.get_tensor_by_name(k)
            if k is g.on_train:
                on_train = bool(v)
            elif isinstance(k, Placeholder) and k.sparse:
                sparse[k] = v
            elif isinstance(k, _Component):
                parts.setdefault(k.parent, {})[k.part] = v
            else:
                raise KeyError(f"cannot feed {k!r}")
        for ph, d in parts.items():
            if set(d) != {"indices", "values", "shape"}:
                raise ValueError(f"{ph.name}: feed indices, values and shape together")
            sparse[ph] = SparseTensorValue(d["indices"], d["values"], d["shape"])
        need = (g.query_batch, g.doc_positive_batch, g.doc_negative_batch)
        missing = [p.name for p in need if p not in sparse]
        if missing:
            raise ValueError(f"missing feeds: {missing}")
        if on_train is None:
            raise ValueError("missing feed: input/on_train")
        q, p, n = (sparse[x] for x in need)
        for sp, rows, nm in ((q, g.query_BS, "query"), (p, g.query_BS, "doc_positive"),
                             (n, g.query_BS * g.NEG, "doc_negative")):
            if int(sp.dense_shape[0]) != rows:
                raise ValueError(f"{nm} batch has {int(sp.dense_shape[0])} rows; the graph's query_BS/NEG "
                                 f"fix it at {rows} (new_dssm.py:131,170)")
            if int(sp.dense_shape[1]) != g.trigram_d:
                raise ValueError(f"{nm} batch width {int(sp.dense_shape[1])} != TRIGRAM_D {g.trigram_d}")
        return feeds_to_csr(q, p, n, g.trigram_d), on_train

    def run(self, fetches, feed_dict: Optional[Dict[Any, Any]] = None):
        g, m = self.graph, self.graph.model
        single = not isinstance(fetches, (list, tuple, dict))
        flat = [fetches] if single else (list(fetches.values()) if isinstance(fetches, dict) else list(fetches))
        flat = [g.get_tensor_by_name(f) if isinstance(f, str) else f for f in flat]
        for f in flat:
            if not isinstance(f, Fetch):
                raise TypeError(f"cannot fetch {f!r}")
        keys = [f.key for f in flat]
        if any(k in _NEEDS_FORWARD for k in keys):
            if not feed_dict:
                raise ValueError("these fetches need the input feeds")
            batch, on_train = self._assemble_feeds(feed_dict)
            if "train_step" in keys and not on_train:
                raise ValueError("train_step needs on_train=True (batch-stat BN); eval-mode training "
                                 "is not a reference configuration")
            m.set_batch(batch)
            if "train_step" in keys:
                m.train_step(self.stream)
            else:
                m.forward(bool(on_train), self.stream)
            torch.cuda.synchronize(m.device)
        out = []
        for k in keys:
            if k == "train_step":
                out.append(None)
            elif k == "auc_op":
                out.append(g.auc.update(dssm_labels(g.query_BS, g.NEG), m.fetch("cos_sim_raw")))
            elif k == "auc_value":
                out.append(g.auc.value())
            else:
                out.append(m.fetch(k))
        if single:
            return out[0]
        if isinstance(fetches, dict):
            return dict(zip(fetches.keys(), out))
        return type(fetches)(out) if isinstance(fetches, tuple) else out


class Saver:
    """tf.train.Saver (new_dssm.py:248,331): params, Adam slots, beta powers and EMA shadows as a
    TF1.x V2 checkpoint under the reference graph's variable names (dssm_amd/tfckpt.py).
    ``save(sess, "model/model_1.ckpt")`` writes model_1.ckpt.index / .data-00000-of-00001 and the
    directory's ``checkpoint`` file and returns the prefix, as TF does; ``restore`` also reads
    the npz form (``format="npz"``)."""

    def __init__(self, format: str = "tf"):
        if format not in ("tf", "npz"):
            raise ValueError("format must be 'tf' or 'npz'")
        self.format = format

    def save(self, sess: Session, save_path: str, write_meta_graph: bool = True) -> str:
        if self.format == "npz" or save_path.endswith(".npz"):
            path = save_path if save_path.endswith(".npz") else save_path + ".npz"
            sess.graph.model.save(path)
            return path
        prefix = tfckpt.save_model(sess.graph.model, save_path)
        if write_meta_graph:
            write_meta(sess.graph, prefix + ".meta")
        return prefix

    def restore(self, sess: Session, save_path: str):
        if os.path.exists(save_path + ".index"):
            tfckpt.restore_model(sess.graph.model, save_path)
            return
        path = save_path if save_path.endswith(".npz") else save_path + ".npz"
        sess.graph.model.restore(path)


# ---- the export script's graph handling (load_model_and_save_vector.py:8-11,25) --------------
# tf.train.Saver.save also writes <prefix>.meta, the MetaGraphDef that import_meta_graph rebuilds the
# graph from.  Here the graph is this module's DSSMGraph, so <prefix>.meta is a JSON description of it
# (the Config fields that shape it and its tensor names), not a protobuf: a TF reader cannot load it,
# and this module's import_meta_graph cannot load a TF one.
META_FORMAT = "dssm_amd.meta/1"
_DEFAULT_GRAPH: Optional[DSSMGraph] = None


def write_meta(graph: DSSMGraph, path: str) -> str:
    with open(path, "w") as f:
        json.dump(graph.meta(), f, indent=1, sort_keys=True)
    return path


def read_meta(path: str) -> Dict[str, Any]:
    with open(path) as f:
        meta = json.load(f)
    if not isinstance(meta, dict) or meta.get("format") != META_FORMAT:
        raise ValueError(f"{path}: not a {META_FORMAT} graph description (a TF MetaGraphDef cannot be "
                         "imported here)")
    return meta


def get_default_graph() -> DSSMGraph:
    """tf.get_default_graph(): the last DSSMGraph built or imported."""
    if _DEFAULT_GRAPH is None:
        raise RuntimeError("no DSSM graph has been built or imported")
    return _DEFAULT_GRAPH


def import_meta_graph(meta_path: str, device=None) -> Saver:
    """tf.train.import_meta_graph (load_model_and_save_vector.py:10): rebuild the graph a
    checkpoint was saved from (it becomes the default graph) and return a Saver for its variables."""
    from .config import Config
    m = read_meta(meta_path)
    conf = Config(query_BS=m["query_BS"], NEG=m["NEG"], L1_N=m["L1_N"], L2_N=m["L2_N"], L3_N=m["L3_N"],
                  learning_rate=m["learning_rate"], compute_dtype=m["compute_dtype"],
                  max_nnz_per_row=m["max_nnz_per_row"], seed=m["seed"])
    DSSMGraph(conf, m["trigram_d"], device=device)
    return Saver()


latest_checkpoint = tfckpt.latest_checkpoint
# the reference reaches these through tf.train
train = SimpleNamespace(Saver=Saver, import_meta_graph=import_meta_graph, latest_checkpoint=latest_checkpoint)


# ---- functional forward ops (inference / export) -----------------------------------------
def _dev_stream(t: torch.Tensor):
    return _lib.stream_ptr(torch.cuda.current_stream(t.device))


def _ldp(n: int) -> int:
    return (n + 7) // 8 * 8


def _wdtype(W: torch.Tensor) -> int:
    if W.dtype == torch.float32:
        return _lib.DSSM_F32
    if W.dtype == torch.bfloat16:
        return _lib.DSSM_BF16
    raise TypeError("weights must be float32 or bfloat16")


def sparse_tensor_dense_matmul(sp, W: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """FC1 (new_dssm.py:124-126): X·W (+ bias) for a SparseTensorValue or a device CSR triple
    (indptr, indices, values).  W: [D x n] contiguous on the device, n a multiple of 4."""
    lib = _lib.load()
    dev = W.device
    if isinstance(sp, SparseTensorValue):
        from .data import coo_to_csr_rows
        ip, ix, vv = coo_to_csr_rows(sp)
        ip, ix, vv = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
                      (ip.astype(np.int32), ix.astype(np.int32), vv.astype(np.float32)))
        if int(sp.dense_shape[1]) != W.shape[0]:
            raise ValueError("sparse width != W rows")
    else:
        ip, ix, vv = sp
    rows, n = ip.numel() - 1, W.shape[1]
    if n % 4 or not W.is_contiguous():
        raise ValueError("W must be contiguous with a multiple-of-4 width")
    Z = torch.empty(rows, _ldp(n), dtype=torch.float32, device=dev)
    b = None if bias is None else bias.to(torch.float32).contiguous()
    _lib.check(lib.dssm_spmm_csr_fwd(_lib.ptr(ip), _lib.ptr(ix), _lib.ptr(vv), rows, _lib.ptr(W), _wdtype(W),
                                     n, n, None if b is None else _lib.ptr(b), _lib.ptr(Z), Z.shape[1],
                                     _dev_stream(W)), "spmm_csr_fwd")
    return Z[:, :n]


def add_layer(inputs: torch.Tensor, in_size: int, out_size: int, activation_function=None,
              weights: Optional[torch.Tensor] = None, biases: Optional[torch.Tensor] = None,
              seed: int = 0):
    """add_layer (README.md:66-76): inputs·W + b, W, b ~ U(-r, r), r = sqrt(6/(in+out)) when not
    given; activation_function None or a callable applied to the device tensor.  Returns
    (outputs, W, b) so the caller owns the new variables (TF would hold them in the graph)."""
    lib = _lib.load()
    dev = inputs.device
    if weights is None:
        rng = np.random.Generator(np.random.PCG64(seed))
        r = np.sqrt(6.0 / (in_size + out_size))
        weights = torch.from_numpy(rng.uniform(-r, r, (in_size, out_size)).astype(np.float32)).to(dev)
        biases = torch.from_numpy(rng.uniform(-r, r, (out_size,)).astype(np.float32)).to(dev)
    if inputs.dtype != weights.dtype:
        raise TypeError("inputs and weights must share a dtype")
    if inputs.shape[1] != in_size or tuple(weights.shape) != (in_size, out_size):
        raise ValueError("shape mismatch")
    if inputs.stride(1) != 1 or weights.stride(1) != 1 or inputs.stride(0) % 4 or weights.stride(0) % 4:
        raise ValueError("row-major inputs/weights with leading dimensions a multiple of 4 required")
    M = inputs.shape[0]
    Z = torch.empty(M, _ldp(out_size), dtype=torch.float32, device=dev)
    b = None if biases is None else biases.to(torch.float32).contiguous()
    _lib.check(lib.dssm_dense_fwd(_lib.ptr(inputs), inputs.stride(0), _lib.ptr(weights), weights.stride(0),
                                  _wdtype(weights), M, in_size, out_size,
                                  None if b is None else _lib.ptr(b), _lib.ptr(Z), Z.shape[1],
                                  _dev_stream(inputs)), "dense_fwd")
    out = Z[:, :out_size]
    if activation_function is not None:
        out = activation_function(out)
    return out, weights, biases


class BatchNormState:
    """The variables batch_normalization creates under variable_scope('bn') (new_dssm.py:73-79):
    beta=0, gamma=1 (trainable), EMA shadows of the batch moments (zero-init, decay 0.5)."""

    def __init__(self, out_size: int, device=None):
        self.gamma = torch.ones(out_size, dtype=torch.float32, device=device)
        self.beta = torch.zeros(out_size, dtype=torch.float32, device=device)
        self.ema_mean = torch.zeros(out_size, dtype=torch.float32, device=device)
        self.ema_var = torch.zeros(out_size, dtype=torch.float32, device=device)
        self._ws = None

    def ws(self, rows: int, ldz: int, device):
        lib = _lib.load()
        nb = int(lib.dssm_bn_ws_bytes(rows, ldz))
        if self._ws is None or self._ws.numel() < nb:
            self._ws = torch.zeros(nb, dtype=torch.uint8, device=device)
        return self._ws


def batch_normalization(x: torch.Tensor, phase_train: bool, out_size: int,
                        state: Optional[BatchNormState] = None, relu: bool = True,
                        eps: float = 1e-3, decay: float = 0.5):
    """batch_normalization (new_dssm.py:62-88) over the rows of one tower, with the ReLU that
    always follows it fused (relu=False for the bare BN).  x: [rows x n] fp32 on the device
    (row stride a multiple of 8).  Returns (out [rows x n] fp32, state)."""
    lib = _lib.load()
    dev = x.device
    if x.dtype != torch.float32 or x.stride(1) != 1 or x.shape[1] != out_size:
        raise ValueError("x must be row-major fp32 [rows x out_size]")
    ldz = x.stride(0)
    if ldz % 8:
        x = torch.nn.functional.pad(x, (0, _ldp(out_size) - out_size)).contiguous()
        ldz = x.stride(0)
    state = state or BatchNormState(out_size, dev)
    rows = x.shape[0]
    out = torch.empty(rows, ldz, dtype=torch.float32, device=dev)
    _lib.check(lib.dssm_bn_relu_fwd(_lib.ptr(x), ldz, rows, out_size, _lib.ptr(state.gamma), _lib.ptr(state.beta),
                                    _lib.ptr(state.ema_mean), _lib.ptr(state.ema_var), float(eps), float(decay),
                                    1 if phase_train else 0, 1 if relu else 0, _lib.ptr(out), _lib.DSSM_F32,
                                    None, None, _lib.ptr(state.ws(rows, ldz, dev)), _dev_stream(x)),
               "bn_relu_fwd")
    return out[:, :out_size], state


def cosine_similarity(query_y: torch.Tensor, doc_positive_y: torch.Tensor, doc_negative_y: torch.Tensor,
                      NEG: int, gamma: float = GAMMA) -> Dict[str, torch.Tensor]:
    """Merge_Negative_Doc + Cosine_Similarity + Loss (new_dssm.py:160-213): returns cos_sim_raw
    [(NEG+1)·BS x 1], cos_sim / prob [BS x (NEG+1)], query_norm_single [BS x 1], loss, accuracy
    and the gradient d loss / d y of every embedding row ([q; pos; neg] order)."""
    lib = _lib.load()
    dev = query_y.device
    BS, n = query_y.shape
    if doc_positive_y.shape != (BS, n) or doc_negative_y.shape != (BS * NEG, n):
        raise ValueError("embedding shapes must be [BS x n], [BS x n], [BS*NEG x n]")
    ld = _ldp(n)
    y = torch.zeros(BS * (2 + NEG), ld, dtype=torch.float32, device=dev)
    y[:BS, :n] = query_y
    y[BS:2 * BS, :n] = doc_positive_y
    y[2 * BS:, :n] = doc_negative_y
    K = NEG + 1
    cos_raw = torch.empty(K * BS, dtype=torch.float32, device=dev)
    cos_sim = torch.empty(BS, K, dtype=torch.float32, device=dev)
    prob = torch.empty(BS, K, dtype=torch.float32, device=dev)
    qn = torch.empty(BS, dtype=torch.float32, device=dev)
    loss = torch.empty(2, dtype=torch.float32, device=dev)
    dy = torch.empty_like(y)
    ws = torch.zeros(2 * ((BS + 3) // 4) + 64, dtype=torch.float32, device=dev)
    _lib.check(lib.dssm_cosine_softmax_loss(_lib.ptr(y), ld, n, BS, NEG, float(gamma), _lib.ptr(cos_raw),
                                            _lib.ptr(cos_sim), _lib.ptr(prob), _lib.ptr(qn), _lib.ptr(loss),
                                            _lib.ptr(dy), _lib.ptr(ws), _dev_stream(y)), "cosine_softmax_loss")
    return {"cos_sim_raw": cos_raw.view(K * BS, 1), "cos_sim": cos_sim, "prob": prob,
            "query_norm_single": qn.view(BS, 1), "loss": loss[0], "accuracy": loss[1],
            "dy": dy[:, :n]}
