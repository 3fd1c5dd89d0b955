"""Generate tests/golden/ref_vectorizer.npz: the vectorizer file format pinned against the
REFERENCE's own ``save_vectorizer`` / ``load_vectorizer`` (utils/utils.py:241-261).

Run in the build container (the reference checkout and python3.9 + scikit-learn 0.24.2 exist only
here; the GPU box has neither and nothing there reads this script):

    PYTHONHASHSEED=0 /opt/conda/bin/python3.9 tests/golden/make_ref_vectorizer.py [/root/reference]

Inputs are the cleaned query / doc / negative texts of tests/golden/ref_feed.npz (themselves the
reference's ``get_data_set_comment`` output).  Two directions are checked here and stored:

1. reference -> build: ``CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b")`` fitted as
   new_dssm.py:37-38 does and written by the reference's ``save_vectorizer``; the file's bytes are
   stored (``ref_pickle``) so the CPU tests can read them with dssm_amd's allow-list loader and
   compare features and counts.
2. build -> reference: the bytes ``dssm_amd.vecpickle.dumps_count_vectorizer`` writes for the
   same vocabulary (that module is pure Python and imports nothing from the build's GPU side) are
   read back by the reference's ``load_vectorizer``; its ``get_feature_names`` and ``transform`` of
   every text must equal the natively fitted vectorizer's, or this script fails.  The verified bytes
   are stored (``ours_pickle``): the CPU test requires the writer to still produce exactly them.

Stand-ins for modules the reference imports at top level but these functions never use:
``tensorflow`` (only ``SparseTensorValue``) and ``jieba`` (empty), as in make_ref_feed.py.
"""
from __future__ import annotations

import collections
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))


def main(ref_root: str) -> None:
    stv = collections.namedtuple("SparseTensorValue", ["indices", "values", "dense_shape"])
    tf_stub = types.ModuleType("tensorflow")
    tf_stub.SparseTensorValue = stv
    sys.modules["tensorflow"] = tf_stub
    sys.modules["jieba"] = types.ModuleType("jieba")
    sys.path.insert(0, ref_root)
    from utils import utils as U  # the reference's own module, unmodified
    from sklearn.feature_extraction.text import CountVectorizer
    import sklearn

    sys.path.insert(0, os.path.join(ROOT, "dssm_amd"))
    import vecpickle  # dssm_amd/vecpickle.py, standalone (no package import: no torch here)

    with np.load(os.path.join(HERE, "ref_feed.npz"), allow_pickle=False) as z:
        query, doc, doc_neg = ([str(s) for s in z[k]] for k in ("query", "doc", "doc_neg"))
    texts = doc + query + doc_neg  # new_dssm.py:37-38 order
    vec = CountVectorizer(token_pattern=r"(?u)\b\w+\b")
    vec.fit(texts)
    names = vec.get_feature_names()
    want = vec.transform(texts)
    with tempfile.TemporaryDirectory() as td:
        ref_path = os.path.join(td, "vectorizer_data")
        U.save_vectorizer(vec, ref_path)
        with open(ref_path, "rb") as f:
            ref_pickle = f.read()
        ours = vecpickle.dumps_count_vectorizer(names)
        ours_path = os.path.join(td, "ours")
        with open(ours_path, "wb") as f:
            f.write(ours)
        back = U.load_vectorizer(ours_path)
    assert type(back) is CountVectorizer, type(back)
    assert back.get_feature_names() == names
    got = back.transform(texts)
    assert got.shape == want.shape and (got != want).nnz == 0, "transform differs"
    out = {
        "sklearn_version": np.array([sklearn.__version__]),
        "texts": np.array(texts), "feature_names": np.array(names),
        "indptr": want.indptr, "indices": want.indices, "data": want.data,
        "ref_pickle": np.frombuffer(ref_pickle, np.uint8),
        "ours_pickle": np.frombuffer(ours, np.uint8),
    }
    dst = os.path.join(HERE, "ref_vectorizer.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: {len(names)} features; the reference's load_vectorizer read the build's pickle "
          f"({len(ours)} B) and transformed {len(texts)} texts identically")


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _isolate import in_child, rerun_isolated
    if not in_child():  # the reference's code runs only in a scrubbed, throwaway child (_isolate.py)
        sys.exit(rerun_isolated(__file__, sys.argv[1:]))
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
