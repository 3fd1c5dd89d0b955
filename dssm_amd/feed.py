"""Host data path: raw comment TSV -> sparse feeds -> device CSR.

Mirrors the reference's pipeline with its names:

* ``pre_process`` (utils/utils.py:424-437) and the tokenisation / vocabulary / counting of
  ``CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b")`` (new_dssm.py:37-45) run natively in
  libdssm.so (``dssm_text_clean``, ``dssm_vocab_*``); ``TextVectorizer`` has sklearn's
  fit / transform / get_feature_names / vocabulary_ surface and returns scipy CSR matrices, so
  ``pull_batch`` and ``convert_sparse_matrix_to_sparse_tensor`` (dssm_amd.data) work on them
  unchanged.  ``save_vectorizer`` / ``load_vectorizer`` (utils/utils.py:241-261) write and read
  the reference's file: a pickled scikit-learn CountVectorizer (dssm_amd.vecpickle).
* ``get_data_set_comment`` (utils/utils.py:368-421): TSV lines ``prefix \\t title \\t label \\t mid
  \\t feed_id`` with label '1', one space-separated character per token, NEG negatives per query
  drawn from the other docs (doc != positive, query differs, no repeats).  The reference draws
  them with ``random.random()`` into a ``set`` (order depends on the string hash seed, SURVEY
  Appendix B.3) and can loop forever; here they come from a seeded PCG64 in draw order, and a
  query with too few eligible docs raises.
* ``get_data_by_dssm2`` (utils/data_input.py:53-60,121-161): the alternative BoW loader over a
  fixed character vocabulary (``load_vocab``, ``DataInputConfig``: the attributes it needs from
  dssm_rnn/config.py), float32 CSR query / doc_pos / doc_neg matrices for ``pull_batch``.
* ``Feeder``: the step's combined CSR [q; pos; neg] of batch b assembled from the three CSR
  matrices by a native worker thread into pinned memory and copied on its own HIP stream
  (``dssm_feeder_*``), double-buffered so batch b+1's H2D overlaps step b; ``DSSM.set_batch``
  then points the plan at the device slot (no host synchronisation on the step path).
"""
from __future__ import annotations

import ctypes as C
import json
from typing import List, Sequence

import numpy as np
import scipy.sparse as sps

from . import _lib
from ._lib import check
from .vecpickle import dumps_count_vectorizer, loads_count_vectorizer


def _cstrs(texts: Sequence[str]):
    enc = [t.encode("utf8") for t in texts]
    arr = (C.c_char_p * max(1, len(enc)))(*enc)
    return arr, enc


def pre_process(line):
    """utils/utils.py:424-437 (native)."""
    if line is None:
        return line
    lib = _lib.load()
    b = line.encode("utf8")
    n = C.c_size_t()
    check(lib.dssm_text_clean(b, None, 0, C.byref(n)), "text_clean")
    out = C.create_string_buffer(n.value + 1)
    check(lib.dssm_text_clean(b, out, n.value + 1, C.byref(n)), "text_clean")
    return out.raw[:n.value].decode("utf8")


class TextVectorizer:
    """CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b") for pre_processed text (native)."""

    def __init__(self):
        self.lib = _lib.load()
        h = C.c_void_p()
        check(self.lib.dssm_vocab_create(C.byref(h)), "vocab_create")
        self._h = h
        self._names: List[str] = []

    def __del__(self):
        if getattr(self, "_h", None):
            self.lib.dssm_vocab_destroy(self._h)
            self._h = None

    def fit(self, raw_documents: Sequence[str]):
        arr, _keep = _cstrs(raw_documents)
        check(self.lib.dssm_vocab_fit(self._h, arr, len(raw_documents)), "vocab_fit")
        n = self.lib.dssm_vocab_finalize(self._h)
        if n < 0:
            check(int(n), "vocab_finalize")
        self._names = [self._name(i) for i in range(int(n))]
        return self

    def _name(self, i: int) -> str:
        buf = C.create_string_buffer(256)
        k = self.lib.dssm_vocab_name(self._h, i, buf, 256)
        if k < 0:
            check(k, "vocab_name")
        if k >= 256:
            buf = C.create_string_buffer(k + 1)
            self.lib.dssm_vocab_name(self._h, i, buf, k + 1)
        return buf.raw[:k].decode("utf8")

    def get_feature_names(self) -> List[str]:
        return list(self._names)

    get_feature_names_out = get_feature_names

    @property
    def vocabulary_(self):
        return {t: i for i, t in enumerate(self._names)}

    def transform(self, raw_documents: Sequence[str]) -> sps.csr_matrix:
        n = len(raw_documents)
        arr, _keep = _cstrs(raw_documents)
        indptr = np.zeros(n + 1, np.int64)
        nnz = C.c_int64()
        ip = indptr.ctypes.data_as(C.c_void_p)
        check(self.lib.dssm_vocab_transform(self._h, arr, n, ip, None, None, 0, C.byref(nnz)), "transform")
        indices = np.zeros(max(1, nnz.value), np.int32)
        values = np.zeros(max(1, nnz.value), np.float32)
        check(self.lib.dssm_vocab_transform(self._h, arr, n, ip, indices.ctypes.data_as(C.c_void_p),
                                            values.ctypes.data_as(C.c_void_p), nnz.value,
                                            C.byref(nnz)), "transform")
        k = nnz.value
        return sps.csr_matrix((values[:k], indices[:k], indptr), shape=(n, len(self._names)))

    def fit_transform(self, raw_documents):
        return self.fit(raw_documents).transform(raw_documents)

    # save_vectorizer / load_vectorizer (utils/utils.py:241-261)
    def save(self, path: str, format: str = "pickle"):
        """format="pickle" (default): the reference's file -- a pickled scikit-learn CountVectorizer
        that its load_vectorizer reads (dssm_amd.vecpickle); "json": a feature list."""
        if format == "pickle":
            with open(path, "wb") as f:
                f.write(dumps_count_vectorizer(self._names))
        elif format == "json":
            with open(path, "w", encoding="utf8") as f:
                json.dump({"format": "dssm_amd.TextVectorizer/1", "features": self._names}, f,
                          ensure_ascii=False)
        else:
            raise ValueError("format must be 'pickle' or 'json'")

    @classmethod
    def from_features(cls, features: Sequence[str]) -> "TextVectorizer":
        """A fitted vectorizer whose column i is features[i]."""
        v = cls()
        for name in features:
            check(v.lib.dssm_vocab_add(v._h, name.encode("utf8")), "vocab_add")
        v._names = list(features)
        return v

    @classmethod
    def load(cls, path: str) -> "TextVectorizer":
        """Either format of ``save``: the reference's pickle (read by an allow-list unpickler that
        resolves nothing but the CountVectorizer state, see dssm_amd.vecpickle) or JSON."""
        with open(path, "rb") as f:
            data = f.read()
        if data.lstrip()[:1] == b"{":
            feats = json.loads(data.decode("utf8"))["features"]
        else:
            feats, _params = loads_count_vectorizer(data)
        return cls.from_features(feats)


def save_vectorizer(vectorizer: TextVectorizer, path: str = "output/vectorizer_data"):
    """utils/utils.py:241-249: the pickled CountVectorizer the reference writes."""
    vectorizer.save(path)


def load_vectorizer(path: str = "output/vectorizer_data") -> TextVectorizer:
    """utils/utils.py:252-261 (also reads this module's JSON form)."""
    return TextVectorizer.load(path)


def get_data_set_comment(FileName: str, conf, seed: int = 0, max_draws: int = 100000,
                         negatives: str = "seeded"):
    """utils/utils.py:368-421.  negatives="seeded" (default): seeded, ordered negatives (module
    doc); negatives="reference": the reference's own draw -- ``random.random()`` from Python's
    global generator into a set per query -- so the same ``random.seed`` and PYTHONHASHSEED give
    the reference's exact negatives and order (tests/test_ref_feed.py)."""
    if negatives not in ("seeded", "reference"):
        raise ValueError("negatives must be 'seeded' or 'reference'")
    query, doc = [], []
    with open(FileName, encoding="utf8") as f:
        for line in f.readlines():
            spline = line.split("\t")
            if len(spline) < 3:
                continue
            prefix, title, label, mid, feed_id = spline  # the reference's unpacking (5 fields)
            if label != "1":
                continue
            query.append(" ".join(pre_process(prefix)))
            doc.append(" ".join(pre_process(title)))
    if negatives == "reference":
        return query, doc, sample_negatives_reference(query, doc, conf.NEG, max_draws=max_draws)
    return query, doc, sample_negatives(query, doc, conf.NEG, seed, max_draws)


def sample_negatives(query: Sequence[str], doc: Sequence[str], neg: int, seed: int = 0,
                     max_draws: int = 100000) -> List[str]:
    """NEG negatives per query j, at rows j*NEG .. j*NEG+NEG-1 (utils/utils.py:403-419)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    size = len(doc)
    out: List[str] = []
    for i in range(size):
        picked: List[str] = []
        draws = 0
        while len(picked) < neg:
            r = int(rng.random() * size)
            cand = doc[r]
            if cand != doc[i] and query[i] != query[r] and cand not in picked:
                picked.append(cand)
            draws += 1
            if draws > max_draws:
                raise ValueError(f"query {i}: fewer than NEG={neg} eligible negative docs")
        out.extend(picked)
    return out


def sample_negatives_reference(query: Sequence[str], doc: Sequence[str], neg: int, rng=None,
                               max_draws: int = 100000) -> List[str]:
    """The reference's negative draw (utils/utils.py:403-419) for drop-in reproducibility: per
    query i, uniform ``int(random() * size)`` picks, rejected when the doc equals the positive,
    the query equals query i, or the doc was already picked; the NEG picks are collected in a
    ``set`` and appended in that set's iteration order (hash-seed dependent, SURVEY Appendix
    B.3).  ``rng`` defaults to Python's global ``random`` module.  Raises instead of spinning
    forever when a query has fewer than NEG eligible docs."""
    import random as _random
    rnd = rng if rng is not None else _random
    size = len(doc)
    out: List[str] = []
    for i in range(size):
        picked = set()
        draws = 0
        while len(picked) < neg:
            r = int(rnd.random() * size)
            cand = doc[r]
            if doc[i] != cand and query[i] != query[r] and cand not in picked:
                picked.add(cand)
            draws += 1
            if draws > max_draws:
                raise ValueError(f"query {i}: fewer than NEG={neg} eligible negative docs")
        out.extend(picked)
    return out


# ---- utils/data_input.py: BoW feeds over a fixed vocabulary (the dssm_rnn configs) -----------
def load_vocab(file_path: str) -> dict:
    """dssm_rnn/config.py:5-11: token -> line number of a vocabulary file (data/vocab.txt)."""
    word_dict = {}
    with open(file_path, encoding="utf8") as f:
        for idx, word in enumerate(f.readlines()):
            word_dict[word.strip()] = idx
    return word_dict


class DataInputConfig:
    """The attributes utils/data_input.py reads from its config (dssm_rnn/config.py:26-29,51):
    vocab_map, nwords, unk, pad, max_seq_len."""

    def __init__(self, vocab_path: str = None, vocab_map: dict = None, unk: str = "[UNK]",
                 pad: str = "[PAD]", max_seq_len: int = 10):
        if vocab_map is None:
            vocab_map = load_vocab(vocab_path)
        self.vocab_map = vocab_map
        self.nwords = len(vocab_map)
        self.unk, self.pad, self.max_seq_len = unk, pad, max_seq_len


def convert_seq2bow(query: str, conf: DataInputConfig) -> dict:
    """utils/data_input.py:53-60: character counts over the vocabulary, out-of-vocabulary
    characters counted at [UNK]; returned sparse ({id: count}) instead of an nwords-long vector."""
    vm, unk = conf.vocab_map, conf.vocab_map[conf.unk]
    out = {}
    for w in query:
        i = vm.get(w, unk)
        out[i] = out.get(i, 0) + 1
    return out


def _bow_csr(rows, nwords: int) -> sps.csr_matrix:
    """float32 CSR of {id: count} rows, column indices ascending (the layout csr_matrix gives the
    reference's dense rows)."""
    indptr = np.zeros(len(rows) + 1, np.int32)
    idx, val = [], []
    for r, d in enumerate(rows):
        ks = sorted(d)
        idx.extend(ks)
        val.extend(d[k] for k in ks)
        indptr[r + 1] = len(idx)
    return sps.csr_matrix((np.asarray(val, np.float32), np.asarray(idx, np.int32), indptr),
                          shape=(len(rows), nwords))


def get_data_by_dssm2(file_path: str, conf: DataInputConfig) -> dict:
    """utils/data_input.py:121-161: TSV lines ``prefix \t query_prediction (JSON) \t title \t tag
    \t label``; label '0' lines are skipped; the negatives are the predicted queries other than the
    title (iteration order of the JSON object), and a line is kept only with at least 4 of them, of
    which the first 4 are used.  Returns {'query', 'doc_pos', 'doc_neg'}: float32 CSR count matrices
    over conf.nwords columns, doc_neg rows 4j..4j+3 belonging to query j -- the matrices pull_batch
    (dssm_amd.data) slices."""
    q, pos, neg = [], [], []
    with open(file_path, encoding="utf8") as f:
        for line in f:
            spline = line.strip().split("\t")
            if len(spline) < 4:
                continue
            prefix, query_pred, title, tag, label = spline
            if label == "0":
                continue
            cur = [convert_seq2bow(each, conf) for each in json.loads(query_pred) if each != title]
            if len(cur) >= 4:
                q.append(convert_seq2bow(prefix, conf))
                pos.append(convert_seq2bow(title, conf))
                neg.extend(cur[:4])
    return {"query": _bow_csr(q, conf.nwords), "doc_pos": _bow_csr(pos, conf.nwords),
            "doc_neg": _bow_csr(neg, conf.nwords)}


class Feeder:
    """Pinned, double-buffered, asynchronous H2D feed of the step's combined CSR (module doc).

    query, doc, doc_neg: scipy CSR matrices ([N x D], [N x D], [N*NEG x D]).  ``start(b)`` queues
    batch b; ``next(model, b_next)`` points the model at the queued batch's device slot (its
    stream waits for the copy on the device), queues b_next into the other slot and returns the
    batch index now set; call ``done(model)`` after the step is enqueued."""

    def __init__(self, query, doc, doc_neg, query_bs: int, neg: int, max_nnz: int, nslots: int = 2):
        self.lib = _lib.load()
        mats = [sps.csr_matrix(m) for m in (query, doc, doc_neg)]
        self._ip = [np.ascontiguousarray(m.indptr, np.int64) for m in mats]
        self._ix = [np.ascontiguousarray(m.indices, np.int32) for m in mats]
        self._vv = [np.ascontiguousarray(m.data, np.float32) for m in mats]
        rows = (C.c_int64 * 3)(*[m.shape[0] for m in mats])
        P3 = C.c_void_p * 3
        h = C.c_void_p()
        check(self.lib.dssm_feeder_create(P3(*[a.ctypes.data for a in self._ip]),
                                          P3(*[a.ctypes.data for a in self._ix]),
                                          P3(*[a.ctypes.data for a in self._vv]), rows, int(query_bs),
                                          int(neg), int(max_nnz), int(nslots), C.byref(h)), "feeder_create")
        self._h = h
        self.nslots = nslots
        self.n_batches = min(mats[0].shape[0] // query_bs, mats[1].shape[0] // query_bs,
                             mats[2].shape[0] // (query_bs * neg))
        self._slot = 0
        self._cur = None
        self._queued = {}

    def close(self):
        if getattr(self, "_h", None):
            self.lib.dssm_feeder_destroy(self._h)
            self._h = None

    __del__ = close

    def start(self, batch: int):
        check(self.lib.dssm_feeder_submit(self._h, self._slot, int(batch)), "feeder_submit")
        self._queued[self._slot] = int(batch)

    def next(self, model, next_batch=None, stream=None) -> int:
        slot = self._slot
        if slot not in self._queued:
            raise RuntimeError("no batch queued: call start(b) first")
        ip, ix, vv = C.c_void_p(), C.c_void_p(), C.c_void_p()
        nnz = C.c_int64()
        check(self.lib.dssm_feeder_acquire(self._h, slot, _lib.stream_ptr(stream), C.byref(ip), C.byref(ix),
                                           C.byref(vv), C.byref(nnz)), "feeder_acquire")
        check(self.lib.dssm_plan_set_batch(model._plan, ip, ix, vv), "set_batch")
        model._batch_refs = (self,)
        b = self._queued.pop(slot)
        self._cur = slot
        self._slot = (slot + 1) % self.nslots
        if next_batch is not None:
            self.start(next_batch)
        return b

    def done(self, stream=None):
        """After the step reading the current slot is enqueued on `stream`."""
        if self._cur is not None:
            check(self.lib.dssm_feeder_release(self._h, self._cur, _lib.stream_ptr(stream)), "feeder_release")
