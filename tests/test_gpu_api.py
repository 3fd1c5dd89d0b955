"""The reference-API mirror (dssm_amd/api.py) driven like new_dssm.py drives TF.

The loop has the shape of new_dssm.py:256-331. It:

* feeds `pull_batch` dicts built from scipy CSR matrices;
* fetches `train_step` / `loss` / `auc_op` / `auc_value`;
* exports embeddings by tensor name with component feeds (load_model_and_save_vector.py:30-73);
* saves and restores a checkpoint.

Every number is checked against the CPU oracle on the same inputs. The functional ops are checked
the same way: `sparse_tensor_dense_matmul`, `add_layer`, `batch_normalization` and
`cosine_similarity`.

Tolerances are fp32 mode: loss rel 1e-5, cosines/probabilities 1e-5 abs, activations 1e-4 rel.
"""
import numpy as np
import pytest
import scipy.sparse as sps
import torch

from dssm_amd import api
from dssm_amd.config import Config
from dssm_amd.data import ZipfColumns, pull_batch, synth_rows
from oracle import dssm_oracle as O

pytestmark = pytest.mark.gpu

D, BS, NEG = 500, 32, 4


def _matrices(n_batches, seed=5):
    cols = ZipfColumns(D)
    rng = np.random.Generator(np.random.PCG64(seed))
    mats = []
    for rows in (n_batches * BS, n_batches * BS, n_batches * BS * NEG):
        ip, ix, vv = synth_rows(rng, cols, rows, 16.0)
        mats.append(sps.csr_matrix((vv, ix, ip), shape=(rows, D)))
    return mats


def _graph(dtype="fp32"):
    conf = Config(query_BS=BS, L1_N=64, L2_N=32, NEG=NEG, learning_rate=0.01, compute_dtype=dtype,
                  max_nnz_per_row=96)
    g = api.DSSMGraph(conf, D)
    cfg = O.OracleConfig(trigram_d=D, widths=[64, 32], query_bs=BS, neg=NEG)
    return conf, g, cfg


def _oracle_state(g, cfg):
    p = {k: v.detach().cpu().numpy().copy() for k, v in g.model.named_params().items()}
    ema = {k: v.detach().cpu().numpy().copy() for k, v in g.model.named_ema().items()}
    return p, ema


def _feed_batch(feed, g):
    from dssm_amd.data import feeds_to_csr
    b = feeds_to_csr(feed[g.query_batch], feed[g.doc_positive_batch], feed[g.doc_negative_batch], D)
    return b.as_dict()


def test_reference_training_loop_and_eval():
    conf, g, cfg = _graph()
    q, d, n = _matrices(3)
    sess = api.Session(g)
    for batch_id in (2, 0, 1):
        feed = pull_batch(True, q, d, n, batch_id, BS, g.query_batch, g.doc_positive_batch,
                          g.doc_negative_batch, g.on_train, conf)
        p, ema = _oracle_state(g, cfg)
        ref, _ = O.forward(cfg, p, ema, _feed_batch(feed, g), True, np.float64)
        _, loss_v = sess.run([g.train_step, g.loss], feed_dict=feed)  # loss of this step's forward
        assert abs(loss_v - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert g.model.global_step == 3
    # eval (on_train=False): EMA-BN forward, loss, auc_op / auc_value
    p, ema = _oracle_state(g, cfg)
    state = None
    for i in range(3):
        feed = pull_batch(False, q, d, n, i, BS, g.query_batch, g.doc_positive_batch,
                          g.doc_negative_batch, g.on_train, conf)
        ref = O.forward_eval_loss(cfg, p, ema, _feed_batch(feed, g))
        loss_v = sess.run(g.loss, feed_dict=feed)
        assert abs(loss_v - ref["loss"]) <= 1e-5 * abs(ref["loss"])
        np.testing.assert_allclose(sess.run(g.cos_sim_raw, feed_dict=feed).ravel(), ref["cos_sim_raw"],
                                   rtol=1e-4, atol=1e-5)
        sess.run(g.auc_op, feed_dict=feed)
        ref_auc, state = O.auc_streaming(np.array([1] * BS + [0] * BS * NEG), ref["cos_sim_raw"], 2000, state)
        auc_v = sess.run(g.auc_value, feed_dict=feed)
        assert abs(auc_v - ref_auc) <= 1e-3, (auc_v, ref_auc)
    # EMA and params did not move in eval
    p2, ema2 = _oracle_state(g, cfg)
    for k in p:
        np.testing.assert_array_equal(p[k], p2[k])
    for k in ema:
        np.testing.assert_array_equal(ema[k], ema2[k])


def test_export_by_tensor_name_and_saver(tmp_path):
    conf, g, cfg = _graph()
    q, d, n = _matrices(1)
    sess = api.Session(g)
    feed = pull_batch(True, q, d, n, 0, BS, g.query_batch, g.doc_positive_batch, g.doc_negative_batch,
                      g.on_train, conf)
    sess.run(g.train_step, feed_dict=feed)
    path = api.Saver().save(sess, str(tmp_path / "model_1.ckpt"))
    saved = g.model.params.cpu().numpy().copy()
    # export path of load_model_and_save_vector.py: tensors by name, component feeds
    get = g.get_tensor_by_name
    comp_feed = {get("input/on_train:0"): False}
    for ph, X in (("query_batch", q), ("doc_positive_batch", d), ("doc_negative_batch", n)):
        from dssm_amd.data import convert_sparse_matrix_to_sparse_tensor
        sv = convert_sparse_matrix_to_sparse_tensor(X)
        comp_feed[get(f"input/{ph}/indices:0")] = sv[0]
        comp_feed[get(f"input/{ph}/values:0")] = sv[1]
        comp_feed[get(f"input/{ph}/shape:0")] = sv[2]
    y = sess.run(get("BN2/embedding_query_y:0"), feed_dict=comp_feed)
    yp = sess.run(get("BN2/embedding_doc_positive_y:0"), feed_dict=comp_feed)
    qn = sess.run(get("Cosine_Similarity/query_norm_single:0"), feed_dict=comp_feed)
    p, ema = _oracle_state(g, cfg)
    feed_eval = dict(feed)
    feed_eval[g.on_train] = False
    ref = O.forward_eval_loss(cfg, p, ema, _feed_batch(feed_eval, g))
    A = ref["layers"][-1]["A"]
    np.testing.assert_allclose(y, A[:BS], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(yp, A[BS:2 * BS], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(qn.ravel(), ref["qn"], rtol=1e-4, atol=1e-6)
    # train further, then restore the checkpoint
    sess.run(g.train_step, feed_dict=feed)
    assert not np.array_equal(g.model.params.cpu().numpy(), saved)
    api.Saver().restore(sess, path)
    np.testing.assert_array_equal(g.model.params.cpu().numpy(), saved)
    assert g.model.global_step == 1
    # feed validation
    bad = dict(feed)
    del bad[g.on_train]
    with pytest.raises(ValueError):
        sess.run(g.loss, feed_dict=bad)
    with pytest.raises(ValueError):
        sess.run(g.train_step, feed_dict={**feed, g.on_train: False})
    with pytest.raises(KeyError):
        get("FC9/nothing:0")


def test_functional_ops_match_oracle():
    dev = torch.device("cuda")
    rng = np.random.Generator(np.random.PCG64(3))
    cols = ZipfColumns(D)
    rows = 96
    ip, ix, vv = synth_rows(rng, cols, rows, 16.0)
    X = sps.csr_matrix((vv, ix, ip), shape=(rows, D))
    from dssm_amd.data import convert_sparse_matrix_to_sparse_tensor
    sv = convert_sparse_matrix_to_sparse_tensor(X)
    W = rng.uniform(-0.1, 0.1, (D, 64)).astype(np.float32)
    b = rng.uniform(-0.1, 0.1, 64).astype(np.float32)
    Wt, bt = torch.from_numpy(W).to(dev), torch.from_numpy(b).to(dev)
    Z = api.sparse_tensor_dense_matmul(sv, Wt, bt)
    Zref = X.astype(np.float64) @ W.astype(np.float64) + b
    np.testing.assert_allclose(Z.cpu().numpy(), Zref, rtol=1e-4, atol=1e-5)
    Zb = api.sparse_tensor_dense_matmul(sv, Wt.to(torch.bfloat16), bt)
    Wb = Wt.to(torch.bfloat16).float().cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(Zb.cpu().numpy(), X.astype(np.float64) @ Wb + b, rtol=1e-4, atol=1e-4)
    # add_layer
    A = torch.relu(Z).contiguous()
    out, W2, b2 = api.add_layer(A, 64, 32, activation_function=torch.relu, seed=4)
    ref = np.maximum(A.cpu().numpy().astype(np.float64) @ W2.cpu().numpy() + b2.cpu().numpy(), 0)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-4, atol=1e-5)
    # batch_normalization: train (batch moments + EMA update), then eval (EMA)
    z = Z.contiguous()
    y, st = api.batch_normalization(z, True, 64)
    zn = z.cpu().numpy().astype(np.float64)
    mu, var = zn.mean(0), ((zn - zn.mean(0)) ** 2).mean(0)
    yref = np.maximum((zn - mu) / np.sqrt(var + 1e-3), 0)
    np.testing.assert_allclose(y.cpu().numpy(), yref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(st.ema_mean.cpu().numpy(), 0.5 * mu, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(st.ema_var.cpu().numpy(), 0.5 * var, rtol=1e-4, atol=1e-6)
    y2, _ = api.batch_normalization(z, False, 64, state=st)
    yref2 = np.maximum((zn - 0.5 * mu) / np.sqrt(0.5 * var + 1e-3), 0)
    np.testing.assert_allclose(y2.cpu().numpy(), yref2, rtol=1e-4, atol=1e-4)
    # cosine_similarity vs the oracle's Merge/Cosine/Loss on the same embeddings
    emb = np.abs(rng.normal(size=(BS * (2 + NEG), 32))).astype(np.float32)
    e = torch.from_numpy(emb).to(dev)
    res = api.cosine_similarity(e[:BS], e[BS:2 * BS], e[2 * BS:], NEG)
    yq, yp, yn = (emb[:BS].astype(np.float64), emb[BS:2 * BS].astype(np.float64), emb[2 * BS:].astype(np.float64))
    docs = [yp] + [yn[k - 1::NEG] for k in range(1, NEG + 1)]
    c = np.stack([(yq * dk).sum(1) / (np.linalg.norm(yq, axis=1) * np.linalg.norm(dk, axis=1)) for dk in docs], 1)
    s = 20 * c
    pr = np.exp(s - s.max(1, keepdims=True))
    pr /= pr.sum(1, keepdims=True)
    np.testing.assert_allclose(res["cos_sim_raw"].cpu().numpy().ravel(), c.T.ravel(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res["prob"].cpu().numpy(), pr, rtol=1e-4, atol=1e-6)
    assert abs(float(res["loss"]) + np.log(pr[:, 0]).mean()) <= 1e-5 * abs(np.log(pr[:, 0]).mean())


def test_sharded_adam_range_updates_only_its_shard():
    """dssm_plan_set_adam_range (the data-parallel zero schedule's optimizer shard): elements
    inside the range step exactly as in the full step, the rest keep their values."""
    from dssm_amd.model import DSSM
    from dssm_amd.data import synth_batch
    D, widths, BS, NEG = 3000, (128, 64), 64, 4
    a = DSSM(D, widths, BS, NEG, dtype="bf16", seed=2)
    b = DSSM(D, widths, BS, NEG, dtype="bf16", seed=2)
    for m in (a, b):
        m.set_fused_w1_adam(False)
        m.set_batch(synth_batch(D, BS, NEG, seed=11, mean_nnz=20))
        m.forward(True)
        m.backward()
    b.grads.copy_(a.grads)  # same gradient (the backward's atomics may differ in the last bits)
    n = a.n_params
    s0, s1 = 64 * 37, 64 * ((n // 64) // 2)
    p0 = b.params.clone()
    a.apply_adam()
    b.set_adam_range(s0, s1)
    b.apply_adam()
    torch.cuda.synchronize()
    assert torch.equal(b.params[s0:s1], a.params[s0:s1])
    assert torch.equal(b.adam_m[s0:s1], a.adam_m[s0:s1])
    assert torch.equal(b.params[:s0], p0[:s0]) and torch.equal(b.params[s1:], p0[s1:])
    assert not torch.any(b.adam_v[s1:n] != 0)
    assert a.beta_powers() == b.beta_powers()
    with pytest.raises(Exception):
        b.set_adam_range(3, 64)  # not 4-aligned
    b.set_fused_w1_adam(True)
    with pytest.raises(Exception):
        b.apply_adam()  # a shard range needs the fused W1 Adam off


def test_export_mid_vectors_eval(tmp_path):
    """load_model_and_save_vector.py end to end: EMA-BN eval forward on the device, the three
    mid-vector files in the reference's text format, values = the oracle's eval embeddings."""
    from dssm_amd.export import export_mid_vectors, mid_vector_line
    conf, g, cfg = _graph()
    conf.query_mid_vector_file = str(tmp_path / "y.txt")
    conf.doc_pos_y_mid_vector_file = str(tmp_path / "dp.txt")
    conf.doc_neg_y_mid_vector_file = str(tmp_path / "dn.txt")
    q, d, n = _matrices(1)
    sess = api.Session(g)
    feed = pull_batch(True, q, d, n, 0, BS, g.query_batch, g.doc_positive_batch, g.doc_negative_batch,
                      g.on_train, conf)
    sess.run(g.train_step, feed_dict=feed)
    texts = [[f"q {i}" for i in range(BS)], [f"d {i}" for i in range(BS)],
             [f"n {i}" for i in range(BS * NEG)]]
    out = export_mid_vectors(sess, g, {k: v for k, v in feed.items() if k is not g.on_train},
                             *texts, conf)
    p, ema = _oracle_state(g, cfg)
    feed_eval = dict(feed)
    feed_eval[g.on_train] = False
    A = O.forward_eval_loss(cfg, p, ema, _feed_batch(feed_eval, g))["layers"][-1]["A"]
    y_dev = g.model.fetch("embedding_all")
    np.testing.assert_allclose(y_dev, A, rtol=1e-4, atol=1e-5)
    for path, tx, rows in ((conf.query_mid_vector_file, texts[0], y_dev[:BS]),
                           (conf.doc_pos_y_mid_vector_file, texts[1], y_dev[BS:2 * BS]),
                           (conf.doc_neg_y_mid_vector_file, texts[2], y_dev[2 * BS:])):
        lines = open(path, encoding="utf8").read().splitlines()
        assert lines == [mid_vector_line(t, r) for t, r in zip(tx, rows)]
        assert out[path] == len(tx)


def test_export_script_sequence_with_meta_graph(tmp_path):
    """load_model_and_save_vector.py:8-46 as written against `tf`, with `tf` = dssm_amd.api:
    Session(), train.import_meta_graph(<prefix>.meta), restore(sess, train.latest_checkpoint(dir)),
    get_default_graph().get_tensor_by_name(...) -- the embeddings equal the saving graph's."""
    conf, g, cfg = _graph()
    q, d, n = _matrices(1)
    sess = api.Session(g)
    feed = pull_batch(True, q, d, n, 0, BS, g.query_batch, g.doc_positive_batch, g.doc_negative_batch,
                      g.on_train, conf)
    sess.run(g.train_step, feed_dict=feed)
    prefix = api.Saver().save(sess, str(tmp_path / "model_1.ckpt"))
    assert (tmp_path / "model_1.ckpt.meta").exists()
    want = sess.run(g.embedding_query_y, feed_dict={**feed, g.on_train: False})
    # the export script, in a fresh graph
    tf = api
    saver = tf.train.import_meta_graph(str(tmp_path / "model_1.ckpt.meta"))
    sess2 = tf.Session()
    saver.restore(sess2, tf.train.latest_checkpoint(str(tmp_path)))
    graph = tf.get_default_graph()
    assert graph is not g and sess2.graph is graph
    get = graph.get_tensor_by_name
    from dssm_amd.data import convert_sparse_matrix_to_sparse_tensor
    f2 = {get("input/on_train:0"): False}
    for ph, X in (("query_batch", q), ("doc_positive_batch", d), ("doc_negative_batch", n)):
        sv = convert_sparse_matrix_to_sparse_tensor(X)
        f2[get(f"input/{ph}/indices:0")] = sv[0]
        f2[get(f"input/{ph}/values:0")] = sv[1]
        f2[get(f"input/{ph}/shape:0")] = sv[2]
    y = sess2.run(get("BN2/embedding_query_y:0"), feed_dict=f2)
    np.testing.assert_array_equal(y, want)
    assert prefix == tf.train.latest_checkpoint(str(tmp_path))
