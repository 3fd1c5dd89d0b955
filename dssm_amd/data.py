"""Host-side feed layer: synthetic trigram batches and the reference's feed contract.

The reference feeds each step with three ``SparseTensorValue`` COO triples built by
``pull_batch`` (utils/utils.py:45-61) from row slices of scipy CSR matrices
(``convert_sparse_matrix_to_sparse_tensor``, utils/utils.py:20-24).  The device path
consumes ONE combined CSR over the step's rows, ordered

    [ query (BS) ; doc_positive (BS) ; doc_negative (BS*NEG, negative i of query j at j*NEG+i) ]

which is exactly the row order the reference's BN towers and Merge_Negative_Doc assume
(new_dssm.py:130, :169-179; negatives per query are contiguous, utils/utils.py:403-419).

Synthetic inputs follow SURVEY.md §8(d): row nnz ~ clip(Poisson(32), 4, 96) distinct
columns, column ids Zipf(a=1.1) over D through a fixed random permutation (seed 1),
values = counts {1,2,3} with P = .85/.12/.03 stored as float32.
"""
from __future__ import annotations

import collections
import dataclasses
from typing import Optional

import numpy as np

# Same field names as tf.SparseTensorValue so feeds built by the reference's pull_batch
# (or by ours) are interchangeable.
SparseTensorValue = collections.namedtuple("SparseTensorValue", ["indices", "values", "dense_shape"])


@dataclasses.dataclass
class CSRBatch:
    """Combined CSR of one step: rows = BS*(2+NEG)."""
    indptr: np.ndarray   # int32 [rows+1]
    indices: np.ndarray  # int32 [nnz]
    values: np.ndarray   # float32 [nnz]
    rows: int
    trigram_d: int

    @property
    def nnz(self) -> int:
        return int(self.indptr[-1])

    def as_dict(self):
        return {"indptr": self.indptr, "indices": self.indices, "values": self.values}


class ZipfColumns:
    """Column sampler: Zipf(a) ranks over [0, D) mapped through a fixed permutation."""

    def __init__(self, trigram_d: int, a: float = 1.1, perm_seed: int = 1, uniform: bool = False):
        self.d = trigram_d
        self.uniform = uniform
        ranks = np.arange(1, trigram_d + 1, dtype=np.float64)
        w = np.ones_like(ranks) if uniform else ranks ** (-a)
        self.cdf = np.cumsum(w / w.sum())
        self.cdf[-1] = 1.0
        self.perm = np.random.Generator(np.random.PCG64(perm_seed)).permutation(trigram_d).astype(np.int32)

    def sample(self, rng: np.random.Generator, n: int) -> np.ndarray:
        u = rng.random(n)
        return self.perm[np.searchsorted(self.cdf, u, side="right").clip(0, self.d - 1)]


def synth_rows(rng: np.random.Generator, cols: ZipfColumns, rows: int, mean_nnz: float = 32.0,
               lo: int = 4, hi: int = 96):
    """CSR rows with distinct, sorted columns."""
    hi = min(hi, cols.d)
    lo = min(lo, hi)
    k = np.clip(rng.poisson(mean_nnz, size=rows), lo, hi).astype(np.int64)
    indptr = np.zeros(rows + 1, np.int64)
    indptr[1:] = np.cumsum(k)
    indices = np.empty(int(indptr[-1]), np.int32)
    for r in range(rows):
        need = int(k[r])
        got = np.empty(0, np.int32)
        while got.size < need:
            cand = cols.sample(rng, 2 * (need - got.size) + 8)
            got = np.unique(np.concatenate([got, cand]))
            if got.size > need:
                # keep a random subset of the distinct columns, preserving determinism
                got = np.sort(rng.choice(got, size=need, replace=False))
        indices[indptr[r]:indptr[r + 1]] = got
    u = rng.random(indices.size)
    values = np.where(u < 0.85, 1.0, np.where(u < 0.97, 2.0, 3.0)).astype(np.float32)
    return indptr.astype(np.int32), indices, values


def synth_batch(trigram_d: int, query_bs: int, neg: int, seed: int, mean_nnz: float = 32.0,
                uniform: bool = False, cols: Optional[ZipfColumns] = None, lo: int = 4,
                hi: int = 96) -> CSRBatch:
    """One step's combined CSR batch (rows = BS*(2+NEG)); batch b uses seed 1000+b by convention."""
    cols = cols or ZipfColumns(trigram_d, uniform=uniform)
    rng = np.random.Generator(np.random.PCG64(seed))
    rows = query_bs * (2 + neg)
    indptr, indices, values = synth_rows(rng, cols, rows, mean_nnz, lo, hi)
    return CSRBatch(indptr, indices, values, rows, trigram_d)


# ---------------------------------------------------------------------------------------------
# Reference feed contract (utils/utils.py:20-24, :45-61) — host side, scipy only.
# ---------------------------------------------------------------------------------------------

def convert_sparse_matrix_to_sparse_tensor(X) -> SparseTensorValue:
    """scipy sparse → COO SparseTensorValue(indices [nnz,2] (row, col), values, dense_shape)
    (utils/utils.py:20-24)."""
    coo = X.tocoo()
    indices = np.stack([coo.row, coo.col], axis=1)
    return SparseTensorValue(indices, coo.data, coo.shape)


def pull_batch(on_training, query_data, doc_data, doc_neg_data, batch_idx, BS, query_batch,
               doc_pos_batch, doc_neg_batch, on_train_batch, conf):
    """Row-slice the three CSR matrices for batch ``batch_idx`` and return the feed dict
    keyed by the placeholders (utils/utils.py:45-61)."""
    query_in = query_data[batch_idx * BS:(batch_idx + 1) * BS, :]
    doc_pos_in = doc_data[batch_idx * BS:(batch_idx + 1) * BS, :]
    doc_neg_in = doc_neg_data[batch_idx * BS * conf.NEG:(batch_idx + 1) * BS * conf.NEG, :]
    return {query_batch: convert_sparse_matrix_to_sparse_tensor(query_in),
            doc_pos_batch: convert_sparse_matrix_to_sparse_tensor(doc_pos_in),
            doc_neg_batch: convert_sparse_matrix_to_sparse_tensor(doc_neg_in),
            on_train_batch: on_training}


def coo_to_csr_rows(stv: SparseTensorValue):
    """One COO SparseTensorValue → (indptr, indices, values) for its rows."""
    idx = np.asarray(stv.indices)
    rows = int(stv.dense_shape[0])
    vals = np.asarray(stv.values, dtype=np.float32)
    if idx.size == 0:
        return np.zeros(rows + 1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32)
    r = idx[:, 0].astype(np.int64)
    c = idx[:, 1].astype(np.int32)
    order = np.lexsort((c, r))
    r, c, vals = r[order], c[order], vals[order]
    counts = np.bincount(r, minlength=rows)
    indptr = np.zeros(rows + 1, np.int64)
    indptr[1:] = np.cumsum(counts)
    return indptr.astype(np.int32), c, vals


def feeds_to_csr(query: SparseTensorValue, doc_pos: SparseTensorValue, doc_neg: SparseTensorValue,
                 trigram_d: Optional[int] = None) -> CSRBatch:
    """Concatenate the three feeds into the combined CSR the device path consumes."""
    parts = [coo_to_csr_rows(s) for s in (query, doc_pos, doc_neg)]
    d = trigram_d if trigram_d is not None else int(query.dense_shape[1])
    indptr = [np.zeros(1, np.int64)]
    off = 0
    for ip, _, _ in parts:
        indptr.append(ip[1:].astype(np.int64) + off)
        off += int(ip[-1])
    indptr = np.concatenate(indptr).astype(np.int32)
    indices = np.concatenate([p[1] for p in parts]).astype(np.int32)
    values = np.concatenate([p[2] for p in parts]).astype(np.float32)
    return CSRBatch(indptr, indices, values, int(indptr.size - 1), d)


def csr_rows_slice(batch: CSRBatch, r0: int, r1: int) -> CSRBatch:
    s, e = int(batch.indptr[r0]), int(batch.indptr[r1])
    return CSRBatch((batch.indptr[r0:r1 + 1] - s).astype(np.int32), batch.indices[s:e].copy(),
                    batch.values[s:e].copy(), r1 - r0, batch.trigram_d)


def shard_batch(batch: CSRBatch, query_bs: int, neg: int, rank: int, world: int) -> CSRBatch:
    """Data-parallel shard by query: rank r takes queries [r*b, (r+1)*b), their
    positives and their NEG negatives, re-laid out as a local [q; pos; neg] batch."""
    assert query_bs % world == 0
    b = query_bs // world
    q0, q1 = rank * b, (rank + 1) * b
    q = csr_rows_slice(batch, q0, q1)
    p = csr_rows_slice(batch, query_bs + q0, query_bs + q1)
    n = csr_rows_slice(batch, 2 * query_bs + q0 * neg, 2 * query_bs + q1 * neg)
    indptr = np.concatenate([q.indptr, p.indptr[1:] + q.nnz, n.indptr[1:] + q.nnz + p.nnz]).astype(np.int32)
    return CSRBatch(indptr, np.concatenate([q.indices, p.indices, n.indices]),
                    np.concatenate([q.values, p.values, n.values]), b * (2 + neg), batch.trigram_d)
