"""Generate tests/golden/ref_data_input.npz by running the REFERENCE's own utils/data_input.py.

Run in the build container (where the reference checkout and /opt/conda/bin/python3.9 exist; the
GPU box has neither, and nothing there reads this script):

    PYTHONUTF8=1 /opt/conda/bin/python3.9 tests/golden/make_ref_data_input.py [/root/reference]

What runs is the reference's unmodified ``utils/data_input.py``: ``get_data_by_dssm2`` (:121-161)
with ``convert_seq2bow`` (:53-60), then the reference's ``pull_batch`` (utils/utils.py:45-61) over
the three matrices it returns.  data_input.py reads ``conf.vocab_map / nwords / unk`` from a
module-level ``Config()``; the dssm package's Config lacks them, so the
module's ``conf`` is replaced by the reference's own ``semantic_matching/dssm_rnn/config.py``
Config -- the config that defines them, loading ``data/vocab.txt`` (dssm_rnn/config.py:5-11,
26-29) -- constructed with the working directory at dssm_rnn/ so its relative vocabulary path
resolves.  The only stand-ins are the inert ``tensorflow`` (``SparseTensorValue`` namedtuple)
and empty ``jieba`` modules utils/utils.py imports at top level (as in make_ref_feed.py).

Input: a synthetic OPPO-format 5-field TSV (``prefix \\t query_prediction \\t title \\t tag \\t
label``, data/readme.md) written here and stored in the fixture with the vocabulary file's lines:
characters in and out of the vocabulary, predictions equal to the title, lines with fewer than 4
remaining predictions and label-0 lines (both skipped by the reference).
"""
from __future__ import annotations

import collections
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

SEED = 77
N_LINES = 40
BS = 4
NEG = 4
HERE = os.path.dirname(os.path.abspath(__file__))


def synth_tsv(rng: random.Random, vocab) -> str:
    inv = [w for w in vocab if len(w) == 1 and not w.isspace()]
    oov = ["龥", "☃", "\U0001F600", "é", "　", " ", "Ж"]

    def text(k):
        return "".join(rng.choice(inv) if rng.random() < 0.85 else rng.choice(oov) for _ in range(k))

    lines = []
    for i in range(N_LINES):
        prefix, title = text(rng.randrange(2, 9)), text(rng.randrange(2, 12))
        preds = [text(rng.randrange(2, 12)) for _ in range(rng.randrange(3, 9))]
        if rng.random() < 0.4:
            preds.insert(rng.randrange(len(preds) + 1), title)  # excluded from the negatives
        qp = json.dumps({p: f"0.{rng.randrange(10, 99)}" for p in preds}, ensure_ascii=False)
        label = "0" if i % 7 == 3 else "1"
        lines.append(f"{prefix}\t{qp}\t{title}\ttag{i % 5}\t{label}\n")
    return "".join(lines)


def main(ref_root: str) -> None:
    stv = collections.namedtuple("SparseTensorValue", ["indices", "values", "dense_shape"])
    tf_stub = types.ModuleType("tensorflow")
    tf_stub.SparseTensorValue = stv
    sys.modules["tensorflow"] = tf_stub
    sys.modules["jieba"] = types.ModuleType("jieba")
    sys.path.insert(0, ref_root)
    cwd = os.getcwd()
    try:
        os.chdir(os.path.join(ref_root, "semantic_matching", "dssm_rnn"))
        from utils import data_input as DI  # the reference's own module, unmodified
        from utils import utils as U
        from semantic_matching.dssm_rnn.config import Config as RnnConfig
        DI.conf = RnnConfig()  # the config that carries vocab_map / nwords / unk / pad
    finally:
        os.chdir(cwd)
    vocab_lines = open(os.path.join(ref_root, "data", "vocab.txt"), encoding="utf8").read().split("\n")
    tsv = synth_tsv(random.Random(SEED), list(DI.conf.vocab_map))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "oppo.tsv")
        with open(path, "w", encoding="utf8") as f:
            f.write(tsv)
        data = DI.get_data_by_dssm2(path)
    out = {"tsv": np.array([tsv]), "vocab_lines": np.array(vocab_lines), "nwords": np.array([DI.conf.nwords]),
           "bs": np.array([BS]), "neg": np.array([NEG])}
    for k in ("query", "doc_pos", "doc_neg"):
        m = data[k]
        out[f"{k}_indptr"], out[f"{k}_indices"], out[f"{k}_data"] = m.indptr, m.indices, m.data
        out[f"{k}_shape"] = np.array(m.shape)
    conf = types.SimpleNamespace(NEG=NEG)
    nb = data["query"].shape[0] // BS
    out["n_batches"] = np.array([nb])
    for b in range(nb):
        feed = U.pull_batch(True, data["query"], data["doc_pos"], data["doc_neg"], b, BS, "q", "p", "n", "t", conf)
        for key in ("q", "p", "n"):
            v = feed[key]
            out[f"b{b}_{key}_indices"] = np.asarray(v.indices)
            out[f"b{b}_{key}_values"] = np.asarray(v.values)
            out[f"b{b}_{key}_shape"] = np.asarray(v.dense_shape, np.int64)
    dst = os.path.join(HERE, "ref_data_input.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: {data['query'].shape[0]} queries over {DI.conf.nwords} words, {nb} batches")


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _isolate import in_child, rerun_isolated
    if not in_child():  # the reference's code runs only in a scrubbed, throwaway child (_isolate.py)
        sys.exit(rerun_isolated(__file__, sys.argv[1:]))
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
