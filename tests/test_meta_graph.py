"""The `.meta` graph description Saver.save writes beside a checkpoint and import_meta_graph reads
(dssm_amd/api.py; load_model_and_save_vector.py:10): round trip of the JSON form, rejection of
anything else (a TF MetaGraphDef included), and the tf.train names the export script calls.  CPU
only: building the graph itself needs the device (tests/test_gpu_api.py)."""
import json

import pytest

from dssm_amd import api


class _FakeGraph:
    def meta(self):
        return {"format": api.META_FORMAT, "trigram_d": 500, "query_BS": 32, "NEG": 4, "L1_N": 64, "L2_N": 32,
                "L3_N": None, "learning_rate": 0.01, "compute_dtype": "fp32", "max_nnz_per_row": 96, "seed": 0,
                "tensors": ["BN2/embedding_query_y", "input/on_train"]}


def test_meta_round_trip(tmp_path):
    p = api.write_meta(_FakeGraph(), str(tmp_path / "model_1.ckpt.meta"))
    assert api.read_meta(p) == _FakeGraph().meta()


def test_meta_rejects_other_files(tmp_path):
    bad = tmp_path / "tf.meta"
    bad.write_bytes(b"\x0a\x0b\x12\x00protobuf")  # a MetaGraphDef is binary protobuf
    with pytest.raises((ValueError, UnicodeDecodeError)):
        api.read_meta(str(bad))
    other = tmp_path / "other.meta"
    other.write_text(json.dumps({"format": "something/else"}))
    with pytest.raises(ValueError):
        api.read_meta(str(other))


def test_tf_train_names():
    assert api.train.import_meta_graph is api.import_meta_graph
    assert api.train.latest_checkpoint is api.latest_checkpoint
    assert api.train.Saver is api.Saver
