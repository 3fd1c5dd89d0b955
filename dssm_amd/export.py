"""Embedding export: the reference's load_model_and_save_vector.py.

The reference restores a checkpoint, runs the three embedding tensors and query_norm_single with
`on_train: False` (EMA batch-norm, load_model_and_save_vector.py:30-106), and appends one text line
per row to the mid-vector files (:108-152):

    <text with spaces removed> \\t <index>:<str(value)[0:6]>,<index>:...

listing only the components with str(value) != "0.0" and value > 0.0001 (the values are the float32
embeddings as Python floats: ``y[i].tolist()``).  `export_mid_vectors` runs the eval forward on the
device (one libdssm.so forward, EMA BN) and writes the three files in that format.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np


def mid_vector_line(text: str, vec) -> str:
    """One output line (load_model_and_save_vector.py:112-121)."""
    parts = []
    for index, j in enumerate(np.asarray(vec, dtype=np.float32).tolist()):
        j_s = str(j)
        if j_s != "0.0" and j > 0.0001:
            parts.append(str(index) + ":" + j_s[0:6])
    return text.replace(" ", "") + "\t" + ",".join(parts)


def append_mid_vectors(path: str, texts: Sequence[str], Y) -> int:
    """Append len(texts) lines to `path` (the reference opens its files with 'a+')."""
    Y = np.asarray(Y)
    if len(texts) != Y.shape[0]:
        raise ValueError("one text per embedding row")
    with open(path, "a+", encoding="utf8") as f:
        for t, y in zip(texts, Y):
            f.write(mid_vector_line(t, y) + "\n")
    return len(texts)


def export_mid_vectors(sess, graph, feed: dict, query_text: Sequence[str], doc_text: Sequence[str],
                       doc_neg_text: Sequence[str], conf) -> dict:
    """Run the eval forward once (on_train=False: the EMA shadows) and append the query /
    doc-positive / doc-negative mid-vector files named by conf (config.py:24-26).  `feed` holds
    the three sparse feeds (placeholder -> SparseTensorValue); on_train is forced to False."""
    feed = dict(feed)
    feed[graph.on_train] = False
    y, yp, yn, qn = sess.run([graph.query_y, graph.doc_positive_y, graph.doc_negative_y,
                              graph.query_norm_single], feed_dict=feed)
    out = {}
    for path, texts, emb in ((conf.query_mid_vector_file, query_text, y),
                             (conf.doc_pos_y_mid_vector_file, doc_text, yp),
                             (conf.doc_neg_y_mid_vector_file, doc_neg_text, yn)):
        out[path] = append_mid_vectors(path, texts, emb)
    out["query_norm_single"] = qn
    return out


def read_mid_vectors(path: str) -> Iterable[tuple]:
    """Parse a mid-vector file back into (text, {index: value}) (for checks and downstream use)."""
    with open(path, encoding="utf8") as f:
        for line in f:
            text, _, vec = line.rstrip("\n").partition("\t")
            d = {}
            if vec:
                for kv in vec.split(","):
                    k, v = kv.split(":")
                    d[int(k)] = float(v)
            yield text, d
