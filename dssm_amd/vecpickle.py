"""The reference's vectorizer file format (save_vectorizer / load_vectorizer, utils/utils.py:241-261):
a pickled scikit-learn ``CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b")`` fitted as
new_dssm.py:37-45 does.  Pure Python (no torch, no scikit-learn), so it also runs where the
reference's own interpreter does.

* ``dumps_count_vectorizer(features)`` writes the pickle that ``pickle.dump(vectorizer)`` of a
  fitted scikit-learn 0.24.2 CountVectorizer holds (the reference's environment):
  the class by reference, then its ``__dict__`` -- constructor parameters, ``fixed_vocabulary_``,
  ``stop_words_``, ``vocabulary_`` ({term: column}) and ``_sklearn_version``.  The opcodes are
  emitted directly (protocol 2), so the bytes do not depend on the writing interpreter.
  ``tests/golden/make_ref_vectorizer.py`` loads them with the reference's ``load_vectorizer`` and
  checks its ``transform`` against a natively fitted CountVectorizer.
* ``loads_count_vectorizer(data)`` reads such a pickle with an allow-list unpickler: only the
  CountVectorizer class (bound to an inert state holder), numpy integer / float types and scalars,
  ``set`` / ``frozenset`` and the protocol-0/1 object reconstructor resolve; any other global
  raises ``pickle.UnpicklingError`` before anything is called.  It returns the feature list in
  column order and the vectorizer's parameters.
"""
from __future__ import annotations

import io
import pickle
import struct
from typing import Dict, List, Sequence, Tuple

TOKEN_PATTERN = r"(?u)\b\w+\b"
SKLEARN_VERSION = "0.24.2"  # the reference environment's scikit-learn

# The CountVectorizer parameters the native vectorizer (dssm_vocab_*) implements, in the order
# scikit-learn 0.24.2's __init__ assigns them.
PARAMS = (
    ("input", "content"), ("encoding", "utf-8"), ("decode_error", "strict"), ("strip_accents", None),
    ("preprocessor", None), ("tokenizer", None), ("analyzer", "word"), ("lowercase", True),
    ("token_pattern", TOKEN_PATTERN), ("stop_words", None), ("max_df", 1.0), ("min_df", 1),
    ("max_features", None), ("ngram_range", (1, 1)), ("vocabulary", None), ("binary", False),
)


class _Emitter:
    """Protocol-2 opcodes for the few value types a CountVectorizer state holds."""

    def __init__(self):
        self.b = io.BytesIO()

    def raw(self, x: bytes):
        self.b.write(x)

    def value(self, v):
        w = self.b.write
        if v is None:
            w(b"N")
        elif v is True:
            w(b"\x88")
        elif v is False:
            w(b"\x89")
        elif isinstance(v, int):
            if 0 <= v < 256:
                w(b"K" + struct.pack("<B", v))
            elif 0 <= v < 65536:
                w(b"M" + struct.pack("<H", v))
            elif -2 ** 31 <= v < 2 ** 31:
                w(b"J" + struct.pack("<i", v))
            else:
                raise ValueError(f"integer out of range: {v}")
        elif isinstance(v, float):
            w(b"G" + struct.pack(">d", v))
        elif isinstance(v, str):
            e = v.encode("utf-8", "surrogatepass")
            w(b"X" + struct.pack("<I", len(e)) + e)
        elif isinstance(v, tuple) and len(v) == 2:
            self.value(v[0])
            self.value(v[1])
            w(b"\x86")
        else:
            raise TypeError(f"unsupported value {type(v)}")

    def dict_items(self, items):
        self.raw(b"}(")
        for k, v in items:
            self.value(k)
            self.value(v)
        self.raw(b"u")


def dumps_count_vectorizer(features: Sequence[str]) -> bytes:
    """Pickle bytes of a fitted CountVectorizer whose sorted vocabulary is ``features``."""
    feats = list(features)
    if feats != sorted(feats):
        raise ValueError("CountVectorizer vocabularies are sorted (column i = i-th smallest term)")
    if len(set(feats)) != len(feats):
        raise ValueError("duplicate features")
    e = _Emitter()
    e.raw(b"\x80\x02csklearn.feature_extraction.text\nCountVectorizer\n)\x81")
    e.raw(b"}(")
    for k, v in PARAMS:
        e.value(k)
        e.value(v)
    e.value("dtype")
    e.raw(b"cnumpy\nint64\n")
    e.value("fixed_vocabulary_")
    e.value(False)
    e.value("stop_words_")
    e.raw(b"cbuiltins\nset\n)R")
    e.value("vocabulary_")
    e.dict_items((t, i) for i, t in enumerate(feats))
    e.value("_sklearn_version")
    e.value(SKLEARN_VERSION)
    e.raw(b"ub.")
    return e.b.getvalue()


class _CountVectorizerState:
    """Inert stand-in the allow-list unpickler binds the CountVectorizer class to."""

    def __setstate__(self, state):
        self.state = dict(state)


def _np_global(module: str, name: str):
    import numpy as np
    if name in ("int64", "int32", "int16", "int8", "uint8", "float64", "float32", "intc", "dtype"):
        return getattr(np, name)
    if name == "scalar" and module in ("numpy.core.multiarray", "numpy._core.multiarray"):
        def scalar(dtype, data=b""):
            if not isinstance(dtype, np.dtype) or dtype.kind not in "iuf" or not isinstance(data, bytes):
                raise pickle.UnpicklingError("numpy scalar of a non-numeric dtype")
            return np.frombuffer(data, dtype=dtype, count=1)[0]
        return scalar
    raise pickle.UnpicklingError(f"global {module}.{name} is not allowed")


class _AllowListUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) == ("sklearn.feature_extraction.text", "CountVectorizer"):
            return _CountVectorizerState
        if module in ("numpy", "numpy.core.multiarray", "numpy._core.multiarray"):
            return _np_global(module, name)
        if module in ("builtins", "__builtin__") and name in ("set", "frozenset", "object"):
            return {"set": set, "frozenset": frozenset, "object": object}[name]
        if (module, name) == ("copyreg", "_reconstructor"):
            def _reconstructor(cls, base, state):
                if cls is not _CountVectorizerState or base is not object or state is not None:
                    raise pickle.UnpicklingError("unexpected reconstructor arguments")
                return _CountVectorizerState()
            return _reconstructor
        raise pickle.UnpicklingError(f"global {module}.{name} is not allowed")


def loads_count_vectorizer(data: bytes) -> Tuple[List[str], Dict[str, object]]:
    """(features in column order, parameters) of a pickled CountVectorizer.  Raises ValueError
    when its parameters are not the ones this vectorizer implements (PARAMS)."""
    obj = _AllowListUnpickler(io.BytesIO(data)).load()
    if not isinstance(obj, _CountVectorizerState) or not hasattr(obj, "state"):
        raise ValueError("not a pickled CountVectorizer")
    st = obj.state
    vocab = st.get("vocabulary_")
    if not isinstance(vocab, dict):
        raise ValueError("the pickled CountVectorizer is not fitted (no vocabulary_)")
    params = {k: st.get(k, d) for k, d in PARAMS}
    bad = {k: params[k] for k, d in PARAMS
           if k not in ("input", "encoding", "decode_error", "max_df", "min_df", "max_features", "vocabulary")
           and params[k] != d}
    if bad:
        raise ValueError(f"CountVectorizer parameters differ from the supported ones: {bad}")
    n = len(vocab)
    feats: List[str] = [""] * n
    seen = [False] * n
    for t, i in vocab.items():
        i = int(i)
        if not 0 <= i < n or seen[i]:
            raise ValueError("vocabulary_ indices are not a permutation of 0..n-1")
        feats[i], seen[i] = t, True
    return feats, params
