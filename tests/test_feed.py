"""Native host data path (dssm_amd/feed.py, csrc/feed.hip) against the reference's text pipeline:
pre_process (utils/utils.py:424-437, restated in oracle/text_oracle.py) and scikit-learn's
CountVectorizer(token_pattern=r"(?u)\\b\\w+\\b") (new_dssm.py:37-45) -- bit-exact -- plus the
combined-CSR assembly of pull_batch.  CPU only (the feeder's device copy: tests/test_gpu_feed.py)."""
import numpy as np
import pytest
import scipy.sparse as sps
from sklearn.feature_extraction.text import CountVectorizer

from dssm_amd.data import feeds_to_csr, pull_batch
from dssm_amd.feed import TextVectorizer, get_data_set_comment, pre_process, sample_negatives
from oracle import text_oracle as T

CJK = [chr(c) for c in range(0x4E00, 0x4E00 + 300)] + ["龥", "龦", "　", "，", "１"]
ASCII = list("abcXYZ019 _-,.!?:/%$@&+*()")
EXTRA = ["é", "\U0001F600", "\t", "　", "ａ"]
URLS = ["http://t.cn/AbC12", "https://x.y/z?q=1&r=%2F", "http://", "https:/", "httpx://a",
        "http://中文"]


def _rand_text(rng, n):
    parts = []
    for _ in range(n):
        u = rng.random()
        if u < 0.55:
            parts.append(CJK[rng.integers(len(CJK))])
        elif u < 0.85:
            parts.append(ASCII[rng.integers(len(ASCII))])
        elif u < 0.93:
            parts.append(EXTRA[rng.integers(len(EXTRA))])
        else:
            parts.append(URLS[rng.integers(len(URLS))])
    return "".join(parts)


def test_pre_process_matches_reference():
    rng = np.random.Generator(np.random.PCG64(3))
    cases = ["", "  ", "刘德华 的歌 http://t.cn/x1 好听",
             "https://a.b/c https://a.b/c 重复", "abchttp://x.yDEF",
             "http://a.b/c中文http://a.b/c", *URLS]
    cases += [_rand_text(rng, int(rng.integers(0, 60))) for _ in range(400)]
    for s in cases:
        assert pre_process(s) == T.pre_process(s), repr(s)


def test_vectorizer_matches_sklearn():
    rng = np.random.Generator(np.random.PCG64(4))
    docs = [T.char_split(T.pre_process(_rand_text(rng, int(rng.integers(0, 40))))) for _ in range(300)]
    docs += ["abc DEF 12 中文 x_y", "A a Ab aB", "", "   "]  # multi-char tokens, case folding
    fit_docs, test_docs = docs[:250] + docs[300:], docs[200:]
    ref = CountVectorizer(token_pattern=r"(?u)\b\w+\b").fit(fit_docs)
    ours = TextVectorizer().fit(fit_docs)
    assert ours.get_feature_names() == list(ref.get_feature_names_out())
    assert ours.vocabulary_ == {k: int(v) for k, v in ref.vocabulary_.items()}
    A, B = ref.transform(test_docs), ours.transform(test_docs)
    A.sort_indices()
    assert A.shape == B.shape
    np.testing.assert_array_equal(A.indptr, B.indptr)
    np.testing.assert_array_equal(A.indices, B.indices)
    np.testing.assert_array_equal(A.data.astype(np.float32), B.data)


def test_vectorizer_save_load(tmp_path):
    docs = ["刘 德 华", "a b 华 c"]
    v = TextVectorizer().fit(docs)
    p = tmp_path / "vectorizer_data.json"
    v.save(str(p))
    w = TextVectorizer.load(str(p))
    assert w.get_feature_names() == v.get_feature_names()
    assert (w.transform(docs) != v.transform(docs)).nnz == 0


def test_data_set_comment_and_feed(tmp_path):
    """TSV -> (query, doc, doc_neg) -> vectorizer -> pull_batch feeds -> combined CSR."""
    rng = np.random.Generator(np.random.PCG64(5))
    lines = []
    for i in range(40):
        q = _rand_text(rng, 6).replace("\t", " ") + str(i)
        d = _rand_text(rng, 10).replace("\t", " ") + "标题" + str(i)
        lines.append(f"{q}\t{d}\t1\tmid{i}\tfeed{i}\n")
    lines.insert(3, "short\tline\n")   # < 3 fields: skipped
    lines.insert(5, "p\tt\t0\tm\tf\n")  # label != '1': skipped
    path = tmp_path / "train.txt"
    path.write_text("".join(lines), encoding="utf8")

    class Conf:
        NEG = 4
    q, d, n = get_data_set_comment(str(path), Conf, seed=7)
    assert len(q) == len(d) == 40 and len(n) == 40 * 4
    assert q[0] == T.char_split(T.pre_process(lines[0].split("\t")[0]))
    for j in range(40):  # negatives: not the positive, no repeats
        negs = n[j * 4:(j + 1) * 4]
        assert len(set(negs)) == 4 and d[j] not in negs
    assert n == sample_negatives(q, d, 4, seed=7)  # seeded, ordered
    vec = TextVectorizer().fit(d + q + n)
    Q, Dm, N = vec.transform(q), vec.transform(d), vec.transform(n)
    feed = pull_batch(True, Q, Dm, N, 1, 8, "q", "p", "n", "t", Conf)
    b = feeds_to_csr(feed["q"], feed["p"], feed["n"], len(vec.get_feature_names()))
    ref = sps.vstack([Q[8:16], Dm[8:16], N[32:64]]).tocsr()
    ref.sort_indices()
    np.testing.assert_array_equal(b.indptr, ref.indptr)
    np.testing.assert_array_equal(b.indices, ref.indices)
    np.testing.assert_array_equal(b.values, ref.data.astype(np.float32))


def test_negative_sampling_raises_without_candidates():
    with pytest.raises(ValueError):
        sample_negatives(["a", "a"], ["x", "y"], 1, max_draws=50)
