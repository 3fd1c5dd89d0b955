"""Generate tests/golden/ref_feed.npz by running the REFERENCE's own data path.

Run (in the build container, where the reference checkout and a python3.9 with NumPy 1.26 /
scikit-learn 0.24 exist; the GPU box has neither, and nothing there reads this script):

    PYTHONHASHSEED=0 /opt/conda/bin/python3.9 tests/golden/make_ref_feed.py [/root/reference]

What runs is the reference's unmodified ``utils/utils.py`` imported from the checkout:
``pre_process`` (:424-437), ``get_data_set_comment`` (:368-421), ``convert_sparse_matrix_to_
sparse_tensor`` (:20-24) and ``pull_batch`` (:45-61), plus ``CountVectorizer(token_pattern=
r"(?u)\\b\\w+\\b")`` fitted on ``ad + bhv + ad_neg`` and ``get_feature_names()`` exactly as
new_dssm.py:37-45 does.  Two modules it imports at top level are absent from the image and get
inert stand-ins that the exercised functions only reference, never compute with:
``tensorflow`` provides ``SparseTensorValue`` -- the plain ``(indices, values, dense_shape)``
namedtuple container ``convert_sparse_matrix_to_sparse_tensor`` returns -- and ``jieba`` is
empty (only ``cut_words``, not called here, uses it).  No TensorFlow arithmetic is involved:
the fixture pins the integer / byte work of the feed (cleaned text, vocabulary order, counts,
COO indices and row order, negative order), not the model.

The negatives pass through a ``set`` (utils.py:408-419), so their order depends on the string
hash seed: PYTHONHASHSEED=0 and ``random.seed(SEED)`` make them reproducible; the seeds are
stored in the fixture.  Input is a synthetic comment TSV (written here, stored in the fixture):
Chinese text, ASCII words, digits, punctuation, full-width and non-BMP characters, short links,
plus lines the reference skips (label != '1', fewer than 3 fields).
"""
from __future__ import annotations

import collections
import os
import random
import sys
import tempfile
import types

import numpy as np

SEED = 1234
NEG = 4
BS = 4
N_LINES = 48

HERE = os.path.dirname(os.path.abspath(__file__))


def synth_tsv(rng: random.Random) -> str:
    han = [chr(c) for c in range(0x4E00, 0x4E00 + 400)]
    words = ["DSSM", "mi355x", "Hello", "world", "GPU", "abc", "x1", "Zeta", "test", "ok", "rocm"]
    junk = ["!", "，", "。", "？", "#", "@", " ", "　", "（", "）", "😀", "𠀀", "é", "_", "-"]
    links = ["http://t.cn/A6abcd", "https://weibo.com/1234?x=1&y=2", "http://a.b/c%20d"]

    def text(k):
        parts = []
        for _ in range(k):
            u = rng.random()
            if u < 0.6:
                parts.append(rng.choice(han))
            elif u < 0.75:
                parts.append(rng.choice(words))
            elif u < 0.85:
                parts.append(str(rng.randrange(0, 1000)))
            elif u < 0.97:
                parts.append(rng.choice(junk))
            else:
                parts.append(rng.choice(links))
        return "".join(parts)

    lines = []
    for i in range(N_LINES):
        prefix, title = text(rng.randrange(3, 14)), text(rng.randrange(3, 14))
        label = "1" if i % 11 != 5 else "0"
        lines.append(f"{prefix}\t{title}\t{label}\tmid{i}\tfeed{i}\n")
        if i % 13 == 7:
            lines.append("short\tline\n")  # < 3 fields: skipped by the reference
    return "".join(lines)


def main(ref_root: str) -> None:
    stv = collections.namedtuple("SparseTensorValue", ["indices", "values", "dense_shape"])
    tf_stub = types.ModuleType("tensorflow")
    tf_stub.SparseTensorValue = stv
    sys.modules["tensorflow"] = tf_stub
    sys.modules["jieba"] = types.ModuleType("jieba")
    sys.path.insert(0, ref_root)
    from utils import utils as U  # the reference's own module, unmodified
    from sklearn.feature_extraction.text import CountVectorizer

    tsv = synth_tsv(random.Random(SEED + 1))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "comment.tsv")
        with open(path, "w", encoding="utf8") as f:
            f.write(tsv)
        conf = types.SimpleNamespace(NEG=NEG)
        random.seed(SEED)
        query, doc, doc_neg = U.get_data_set_comment(path, conf)
    fields = [fld for line in tsv.splitlines() for fld in line.split("\t")[:2]]
    cleaned = [U.pre_process(fld) for fld in fields]
    vec = CountVectorizer(token_pattern=r"(?u)\b\w+\b")
    vec.fit(doc + query + doc_neg)  # new_dssm.py:37-38 order: ad_act + bhv_act + ad_act_neg
    names = vec.get_feature_names()
    mats = {k: vec.transform(v) for k, v in (("query", query), ("doc", doc), ("doc_neg", doc_neg))}
    out = {
        "seed": np.array([SEED], np.int64), "hashseed": np.array([int(os.environ.get("PYTHONHASHSEED", -1))]),
        "neg": np.array([NEG], np.int64), "bs": np.array([BS], np.int64),
        "tsv": np.array([tsv]), "fields": np.array(fields), "cleaned": np.array(cleaned),
        "query": np.array(query), "doc": np.array(doc), "doc_neg": np.array(doc_neg),
        "feature_names": np.array(names),
    }
    for k, m in mats.items():
        out[f"{k}_indptr"], out[f"{k}_indices"], out[f"{k}_data"] = m.indptr, m.indices, m.data
    nb = mats["query"].shape[0] // BS
    out["n_batches"] = np.array([nb], np.int64)
    for b in range(nb):
        feed = U.pull_batch(True, mats["query"], mats["doc"], mats["doc_neg"], b, BS, "q", "p", "n", "t", conf)
        for key in ("q", "p", "n"):
            v = feed[key]
            out[f"b{b}_{key}_indices"] = np.asarray(v.indices)
            out[f"b{b}_{key}_values"] = np.asarray(v.values)
            out[f"b{b}_{key}_shape"] = np.asarray(v.dense_shape, np.int64)
    dst = os.path.join(HERE, "ref_feed.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: {len(query)} queries, {len(names)} features, {nb} batches of BS={BS}")


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _isolate import in_child, rerun_isolated
    if not in_child():  # the reference's code runs only in a scrubbed, throwaway child (_isolate.py)
        sys.exit(rerun_isolated(__file__, sys.argv[1:]))
    if os.environ.get("PYTHONHASHSEED") != "0":
        sys.exit("run with PYTHONHASHSEED=0 (the reference orders negatives through a set)")
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
