"""utils/data_input.py's BoW loader against outputs the REFERENCE's own code produced
(tests/golden/ref_data_input.npz, made by tests/golden/make_ref_data_input.py: the reference's
get_data_by_dssm2 / convert_seq2bow (utils/data_input.py:53-60,121-161) run unmodified with the
dssm_rnn Config's vocabulary, then its pull_batch).  Integer / byte work, so every comparison is
exact:
* ``load_vocab`` on the reference's data/vocab.txt lines (stored in the fixture);
* ``get_data_by_dssm2``: the three float32 CSR count matrices (shape, indptr, indices, data);
* ``pull_batch`` over those matrices: every batch's COO feeds, and the combined device CSR."""
import os

import numpy as np
import pytest
import scipy.sparse as sps

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "ref_data_input.npz")


def load_ref():
    with np.load(FIX, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def ref():
    return load_ref()


def ref_matrix(ref, k):
    return sps.csr_matrix((ref[f"{k}_data"], ref[f"{k}_indices"], ref[f"{k}_indptr"]),
                          shape=tuple(int(x) for x in ref[f"{k}_shape"]))


def ref_feeds(ref, b):
    from dssm_amd.data import SparseTensorValue
    return [SparseTensorValue(ref[f"b{b}_{k}_indices"], ref[f"b{b}_{k}_values"], ref[f"b{b}_{k}_shape"])
            for k in ("q", "p", "n")]


def build_data(ref, tmp_path):
    from dssm_amd.feed import DataInputConfig, get_data_by_dssm2
    vocab = tmp_path / "vocab.txt"
    vocab.write_text("\n".join(str(x) for x in ref["vocab_lines"]), encoding="utf8")
    tsv = tmp_path / "oppo.tsv"
    tsv.write_text(str(ref["tsv"][0]), encoding="utf8")
    conf = DataInputConfig(vocab_path=str(vocab))
    return conf, get_data_by_dssm2(str(tsv), conf)


def test_get_data_by_dssm2_matches_reference(ref, tmp_path):
    conf, data = build_data(ref, tmp_path)
    assert conf.nwords == int(ref["nwords"][0])
    assert data["query"].shape[0] >= 4 and data["doc_neg"].shape[0] == 4 * data["query"].shape[0]
    for k in ("query", "doc_pos", "doc_neg"):
        got, want = data[k], ref_matrix(ref, k)
        assert got.shape == want.shape and got.dtype == want.dtype == np.float32, k
        np.testing.assert_array_equal(got.indptr, want.indptr)
        np.testing.assert_array_equal(got.indices, want.indices)
        np.testing.assert_array_equal(got.data, want.data)
    unk = conf.vocab_map[conf.unk]
    assert any(unk in ref_matrix(ref, k).indices for k in ("query", "doc_pos", "doc_neg"))  # OOV exercised


def test_pull_batch_on_data_input_matches_reference(ref, tmp_path):
    from types import SimpleNamespace
    from dssm_amd.data import feeds_to_csr, pull_batch
    _, data = build_data(ref, tmp_path)
    BS, NEG = int(ref["bs"][0]), int(ref["neg"][0])
    conf = SimpleNamespace(NEG=NEG)
    for b in range(int(ref["n_batches"][0])):
        feed = pull_batch(True, data["query"], data["doc_pos"], data["doc_neg"], b, BS, "q", "p", "n", "t", conf)
        for key in ("q", "p", "n"):
            idx = np.asarray(feed[key].indices)
            want = ref[f"b{b}_{key}_indices"]
            assert idx.dtype == want.dtype and idx.shape == want.shape, (b, key)
            np.testing.assert_array_equal(idx, want)
            np.testing.assert_array_equal(np.asarray(feed[key].values), ref[f"b{b}_{key}_values"])
            assert tuple(feed[key].dense_shape) == tuple(ref[f"b{b}_{key}_shape"])
        batch = feeds_to_csr(*ref_feeds(ref, b), trigram_d=int(ref["nwords"][0]))
        want = sps.vstack([data["query"][b * BS:(b + 1) * BS], data["doc_pos"][b * BS:(b + 1) * BS],
                           data["doc_neg"][b * BS * NEG:(b + 1) * BS * NEG]]).tocsr()
        np.testing.assert_array_equal(batch.indptr, want.indptr)
        np.testing.assert_array_equal(batch.indices, want.indices)
        np.testing.assert_array_equal(batch.values, want.data)
