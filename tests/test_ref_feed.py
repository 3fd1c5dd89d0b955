"""The host data path against outputs the REFERENCE's own code produced (tests/golden/ref_feed.npz,
made by tests/golden/make_ref_feed.py: the reference's utils/utils.py run unmodified under
python3.9 + scikit-learn 0.24 on a synthetic comment TSV).  Everything here is integer / byte
work, so every comparison is exact:

* ``pre_process`` (utils/utils.py:424-437) on every TSV field;
* ``get_data_set_comment`` (:368-421): the query / doc lists, and with negatives="reference" the
  reference's negatives in the reference's order (same ``random.seed``, PYTHONHASHSEED=0);
* the vocabulary (get_feature_names order) and the count matrices of
  ``CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b")`` fitted as new_dssm.py:37-45 does;
* ``pull_batch`` / ``convert_sparse_matrix_to_sparse_tensor`` (:20-24, :45-61): COO indices (row
  order, dtype), values and dense shapes of every batch, and the combined device CSR built from
  those feeds.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sps

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FIX = os.path.join(HERE, "golden", "ref_feed.npz")


def load_ref():
    with np.load(FIX, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def ref():
    return load_ref()


def ref_matrix(ref, k):
    n = ref[f"{k}_indptr"].size - 1
    return sps.csr_matrix((ref[f"{k}_data"], ref[f"{k}_indices"], ref[f"{k}_indptr"]),
                          shape=(n, ref["feature_names"].size))


def ref_feeds(ref, b):
    """Batch b's three feeds exactly as the reference's pull_batch returned them."""
    from dssm_amd.data import SparseTensorValue
    return [SparseTensorValue(ref[f"b{b}_{k}_indices"], ref[f"b{b}_{k}_values"], ref[f"b{b}_{k}_shape"])
            for k in ("q", "p", "n")]


def test_pre_process_matches_reference(ref):
    from dssm_amd.feed import pre_process
    got = [pre_process(str(f)) for f in ref["fields"]]
    assert got == [str(c) for c in ref["cleaned"]]


def test_get_data_set_comment_matches_reference(ref, tmp_path):
    path = tmp_path / "comment.tsv"
    path.write_text(str(ref["tsv"][0]), encoding="utf8")
    neg, seed = int(ref["neg"][0]), int(ref["seed"][0])
    code = (
        "import json, random, sys, types\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from dssm_amd.feed import get_data_set_comment\n"
        f"random.seed({seed})\n"
        f"q, d, n = get_data_set_comment({str(path)!r}, types.SimpleNamespace(NEG={neg}), "
        "negatives='reference')\n"
        "print(json.dumps([q, d, n], ensure_ascii=False))\n")
    # the reference orders each query's negatives through a set: same string hash seed
    env = dict(os.environ, PYTHONHASHSEED=str(int(ref["hashseed"][0])))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    q, d, n = json.loads(out.stdout.strip().splitlines()[-1])
    assert q == [str(x) for x in ref["query"]]
    assert d == [str(x) for x in ref["doc"]]
    assert n == [str(x) for x in ref["doc_neg"]]  # same negatives, same (set) order


def test_seeded_negatives_follow_the_reference_rules(ref, tmp_path):
    from types import SimpleNamespace
    from dssm_amd.feed import get_data_set_comment
    path = tmp_path / "comment.tsv"
    path.write_text(str(ref["tsv"][0]), encoding="utf8")
    neg = int(ref["neg"][0])
    q, d, n = get_data_set_comment(str(path), SimpleNamespace(NEG=neg), seed=3)
    assert q == [str(x) for x in ref["query"]] and d == [str(x) for x in ref["doc"]]
    assert len(n) == neg * len(q)
    for i in range(len(q)):
        picks = n[i * neg:(i + 1) * neg]
        assert len(set(picks)) == neg and d[i] not in picks
        assert all(q[d.index(p)] != q[i] for p in picks if d.count(p) == 1)


def test_vectorizer_matches_reference(ref):
    from dssm_amd.feed import TextVectorizer
    q, d, n = ([str(x) for x in ref[k]] for k in ("query", "doc", "doc_neg"))
    v = TextVectorizer().fit(d + q + n)
    assert v.get_feature_names() == [str(x) for x in ref["feature_names"]]
    for k, texts in (("query", q), ("doc", d), ("doc_neg", n)):
        got, want = v.transform(texts), ref_matrix(ref, k)
        np.testing.assert_array_equal(got.indptr, want.indptr)
        np.testing.assert_array_equal(got.indices, want.indices)
        np.testing.assert_array_equal(got.data, want.data)


def test_pull_batch_matches_reference(ref):
    from types import SimpleNamespace
    from dssm_amd.data import feeds_to_csr, pull_batch
    conf = SimpleNamespace(NEG=int(ref["neg"][0]))
    BS = int(ref["bs"][0])
    mats = [ref_matrix(ref, k) for k in ("query", "doc", "doc_neg")]
    for b in range(int(ref["n_batches"][0])):
        feed = pull_batch(True, *mats, b, BS, "q", "p", "n", "t", conf)
        for key in ("q", "p", "n"):
            idx = np.asarray(feed[key].indices)
            want = ref[f"b{b}_{key}_indices"]
            assert idx.dtype == want.dtype and idx.shape == want.shape, (b, key, idx.dtype, want.dtype)
            np.testing.assert_array_equal(idx, want)
            np.testing.assert_array_equal(np.asarray(feed[key].values), ref[f"b{b}_{key}_values"])
            assert tuple(feed[key].dense_shape) == tuple(ref[f"b{b}_{key}_shape"])
        # the combined device CSR from the reference's own COO feeds = the rows [q; pos; neg]
        batch = feeds_to_csr(*ref_feeds(ref, b))
        want = sps.vstack([mats[0][b * BS:(b + 1) * BS], mats[1][b * BS:(b + 1) * BS],
                           mats[2][b * BS * conf.NEG:(b + 1) * BS * conf.NEG]]).tocsr()
        np.testing.assert_array_equal(batch.indptr, want.indptr)
        np.testing.assert_array_equal(batch.indices, want.indices)
        np.testing.assert_array_equal(batch.values, want.data.astype(np.float32))
