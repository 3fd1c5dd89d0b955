"""The vectorizer file format against the REFERENCE's save_vectorizer / load_vectorizer
(utils/utils.py:241-261), via tests/golden/ref_vectorizer.npz (made by
tests/golden/make_ref_vectorizer.py under python3.9 + scikit-learn 0.24.2, the reference's
environment).  That script has already checked the build -> reference direction (the reference's
load_vectorizer read dssm_amd's pickle and transformed every text identically); here:

* the writer still produces exactly the bytes the reference verified;
* the reference's own pickle is read by dssm_amd's allow-list loader: same vocabulary, and the
  native vectorizer built from it counts every text exactly as the reference's did;
* save_vectorizer / load_vectorizer round trips; foreign globals are refused, never called.
"""
import os
import pickle

import numpy as np
import pytest
import scipy.sparse as sps

from dssm_amd import vecpickle

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "ref_vectorizer.npz")


@pytest.fixture(scope="module")
def ref():
    with np.load(FIX, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def test_writer_bytes_are_the_ones_the_reference_loaded(ref):
    names = [str(s) for s in ref["feature_names"]]
    assert vecpickle.dumps_count_vectorizer(names) == ref["ours_pickle"].tobytes()


def test_reference_pickle_reads_back(ref):
    feats, params = vecpickle.loads_count_vectorizer(ref["ref_pickle"].tobytes())
    assert feats == [str(s) for s in ref["feature_names"]]
    assert params["token_pattern"] == vecpickle.TOKEN_PATTERN and params["lowercase"] is True


def test_native_counts_from_reference_pickle(ref, tmp_path):
    from dssm_amd.feed import load_vectorizer
    p = tmp_path / "vectorizer_data"
    p.write_bytes(ref["ref_pickle"].tobytes())
    vec = load_vectorizer(str(p))
    texts = [str(s) for s in ref["texts"]]
    got = vec.transform(texts)
    want = sps.csr_matrix((ref["data"], ref["indices"], ref["indptr"]), shape=got.shape)
    assert vec.get_feature_names() == [str(s) for s in ref["feature_names"]]
    assert (got != want).nnz == 0


def test_save_load_round_trip(tmp_path):
    from dssm_amd.feed import TextVectorizer, load_vectorizer, save_vectorizer
    texts = ["a b c", "b d 中 文", "x1 y2 z3 b"]
    v = TextVectorizer().fit(texts)
    for fmt in ("pickle", "json"):
        p = tmp_path / f"vec_{fmt}"
        if fmt == "pickle":
            save_vectorizer(v, str(p))
        else:
            v.save(str(p), format="json")
        w = load_vectorizer(str(p))
        assert w.get_feature_names() == v.get_feature_names()
        assert (w.transform(texts) != v.transform(texts)).nnz == 0


class _Boom:
    def __reduce__(self):
        return (os.system, ("echo should-not-run",))


@pytest.mark.parametrize("payload", [
    pickle.dumps(_Boom()),
    b"\x80\x02cos\nsystem\nX\x04\x00\x00\x00trueR.",
    pickle.dumps({"vocabulary_": {"a": 0}}),
])
def test_foreign_pickles_refused(payload):
    with pytest.raises((pickle.UnpicklingError, ValueError)):
        vecpickle.loads_count_vectorizer(payload)


def test_unsupported_parameters_refused():
    data = vecpickle.dumps_count_vectorizer(["a", "b"]).replace(b"\x88", b"\x89", 1)  # lowercase=False
    with pytest.raises(ValueError, match="lowercase"):
        vecpickle.loads_count_vectorizer(data)
