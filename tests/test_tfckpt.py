"""TF1.x V2 checkpoint files (dssm_amd/tfckpt.py; tf.train.Saver at new_dssm.py:248,331).

TensorFlow is absent from the image, so no TF reader pins these files (parity unpinned); the
tests pin the pieces against their specifications instead:

* CRC-32C against the standard check value and split-buffer extension, LevelDB's mask / unmask;
* the table layout decoded by an independent reading of the LevelDB format written here (footer
  magic and handles, per-block trailer CRC over contents + type byte, restart array), including
  multi-block indexes and prefix-compressed keys;
* BundleEntryProto / BundleHeaderProto field encodings byte by byte;
* write -> read round trips of float32 / int64 tensors of every rank, corruption detected;
* the variable names of the reference graph (2 layers, config.py:19-28) written out in full.
"""
import os
import struct

import numpy as np
import pytest
import torch

from dssm_amd import tfckpt as T


def test_crc32c_known_answer_and_extend():
    assert T.crc32c(b"123456789") == 0xE3069283
    assert T.crc32c(b"") == 0
    d = np.random.default_rng(0).integers(0, 256, 100003, dtype=np.uint8).tobytes()
    assert T.crc32c(d[50001:], T.crc32c(d[:50001])) == T.crc32c(d)
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert T.unmask(T.mask(c)) == c
    assert T.mask(0) == 0xA282EAD8


def _decode_table(buf):
    """Independent LevelDB table decoder (format spec), returning [(key, value)] in file order."""
    assert struct.unpack("<Q", buf[-8:])[0] == 0xDB4775248B80FB57
    footer = buf[-48:-8]

    def varint(b, i):
        x = s = 0
        while True:
            c = b[i]
            i += 1
            x |= (c & 0x7F) << s
            if c < 0x80:
                return x, i
            s += 7

    mo, i = varint(footer, 0)
    ms, i = varint(footer, i)
    io, i = varint(footer, i)
    isz, i = varint(footer, i)

    def block(off, size):
        body = buf[off:off + size + 1]
        crc = struct.unpack("<I", buf[off + size + 1:off + size + 5])[0]
        assert body[-1] == 0 and T.unmask(crc) == T.crc32c(body)
        c = body[:-1]
        n = struct.unpack("<I", c[-4:])[0]
        restarts = [struct.unpack("<I", c[-4 - 4 * (n - k):-4 - 4 * (n - k) + 4])[0] for k in range(n)]
        end, j, prev, out = len(c) - 4 - 4 * n, 0, b"", []
        while j < end:
            if j in restarts:
                prev = b""
            sh, j = varint(c, j)
            ns, j = varint(c, j)
            vl, j = varint(c, j)
            key = prev[:sh] + c[j:j + ns]
            out.append((key, c[j + ns:j + ns + vl]))
            j += ns + vl
            prev = key
        return out

    assert block(mo, ms) == []
    items = []
    for _k, h in block(io, isz):
        o, j = varint(h, 0)
        s, _ = varint(h, j)
        items += block(o, s)
    return items


def test_table_layout_multi_block():
    rng = np.random.default_rng(1)
    items = {f"layer{i // 7}/var{i:03d}/Adam".encode(): rng.bytes(int(rng.integers(0, 60)))
             for i in range(300)}
    items[b""] = b"hdr"
    buf = T.write_table(items, block_bytes=512)
    got = _decode_table(buf)
    assert [k for k, _ in got] == sorted(items)
    assert dict(got) == items
    assert T.read_table(buf) == items


def test_proto_encodings():
    assert T._header_proto() == b"\x08\x01\x1a\x02\x08\x01"
    e = T._entry_proto(T.DT_FLOAT, (300, 2), 1000, 2400, 0x01020304)
    assert e == (b"\x08\x01" + b"\x12\x09" + b"\x12\x03\x08\xac\x02" + b"\x12\x02\x08\x02"
                 + b"\x20\xe8\x07" + b"\x28\xe0\x12" + b"\x35\x04\x03\x02\x01")
    assert T._parse_entry(e) == {"dtype": 1, "shape": [300, 2], "shard_id": 0, "offset": 1000,
                                 "size": 2400, "crc32c": 0x01020304}
    scalar = T._entry_proto(T.DT_FLOAT, (), 0, 4, 7)
    assert scalar.startswith(b"\x08\x01\x12\x00\x28\x04")


def test_round_trip_and_checkpoint_file(tmp_path):
    rng = np.random.default_rng(2)
    tensors = {"FC1/Variable": rng.standard_normal((50, 7)).astype(np.float32),
               "FC1/Variable_1": rng.standard_normal(7).astype(np.float32),
               "Training/beta1_power": np.array(0.729, np.float32),
               "global_step": np.array(12345678901, np.int64),
               "empty": np.zeros((0, 3), np.float32)}
    prefix = str(tmp_path / "model" / "model_1.ckpt")
    assert T.write_checkpoint(prefix, tensors) == prefix
    assert os.path.getsize(prefix + ".data-00000-of-00001") == sum(a.nbytes for a in tensors.values())
    back = T.read_checkpoint(prefix)
    assert set(back) == set(tensors)
    for k, a in tensors.items():
        assert back[k].dtype == a.dtype and back[k].shape == a.shape and np.array_equal(back[k], a)
    assert T.latest_checkpoint(str(tmp_path / "model")) == prefix
    with open(prefix + ".data-00000-of-00001", "r+b") as f:
        f.seek(3)
        f.write(b"\xff")
    with pytest.raises(ValueError, match="checksum"):
        T.read_checkpoint(prefix)


REFERENCE_NAMES = sorted([
    "FC1/Variable", "FC1/Variable_1", "FC2/Variable", "FC2/Variable_1",
    "BN1/bn/beta", "BN1/bn/gamma", "BN1/bn_1/beta", "BN1/bn_1/gamma",
    "BN2/bn/beta", "BN2/bn/gamma", "BN2/bn_1/beta", "BN2/bn_1/gamma",
    "bn/BN1/bn/moments/Squeeze/ExponentialMovingAverage", "bn/BN1/bn/moments/Squeeze_1/ExponentialMovingAverage",
    "bn/BN1/bn_1/moments/Squeeze/ExponentialMovingAverage", "bn/BN1/bn_1/moments/Squeeze_1/ExponentialMovingAverage",
    "bn/BN2/bn/moments/Squeeze/ExponentialMovingAverage", "bn/BN2/bn/moments/Squeeze_1/ExponentialMovingAverage",
    "bn/BN2/bn_1/moments/Squeeze/ExponentialMovingAverage", "bn/BN2/bn_1/moments/Squeeze_1/ExponentialMovingAverage",
    "Training/beta1_power", "Training/beta2_power",
] + [f"{v}/Adam{s}" for v in ["FC1/Variable", "FC1/Variable_1", "FC2/Variable", "FC2/Variable_1",
                               "BN1/bn/beta", "BN1/bn/gamma", "BN1/bn_1/beta", "BN1/bn_1/gamma",
                               "BN2/bn/beta", "BN2/bn/gamma", "BN2/bn_1/beta", "BN2/bn_1/gamma"]
     for s in ("", "_1")])


class _StubModel:
    """named_params / named_adam / named_ema / beta_powers / load_* of DSSM, on CPU tensors."""

    def __init__(self, D, widths, seed):
        g = torch.Generator().manual_seed(seed)
        self.widths, self.beta1 = list(widths), 0.9
        dims = [D] + self.widths

        def views():
            out = {}
            for l in range(1, len(widths) + 1):
                out[f"W{l}"] = torch.randn(dims[l - 1], dims[l], generator=g)
                out[f"b{l}"] = torch.randn(dims[l], generator=g)
                for t in "qd":
                    for k in ("gamma", "beta"):
                        out[f"bn{l}_{t}_{k}"] = torch.randn(dims[l], generator=g)
            return out

        self.p, self.m, self.v = views(), views(), views()
        self.ema = {f"bn{l}_{t}_{s}": torch.rand(n, generator=g)
                    for l, n in enumerate(self.widths, 1) for t in "qd" for s in ("mean", "var")}
        self.b = (np.float32(0.9 ** 3), np.float32(0.999 ** 3))

    def named_params(self):
        return self.p

    def named_adam(self):
        return self.m, self.v

    def named_ema(self):
        return self.ema

    def beta_powers(self):
        return self.b

    def load_adam_state(self, m, v, b1, b2, step):
        for src, dst in ((m, self.m), (v, self.v)):
            for k, a in src.items():
                dst[k].copy_(torch.from_numpy(np.asarray(a)))
        self.b, self.step = (np.float32(b1), np.float32(b2)), step

    def load_params(self, p, ema=None):
        for k, a in p.items():
            self.p[k].copy_(torch.from_numpy(np.asarray(a)))
        for k, a in (ema or {}).items():
            self.ema[k].copy_(torch.from_numpy(np.asarray(a)))


def test_reference_graph_names_and_model_round_trip(tmp_path):
    src = _StubModel(1000, (100, 100), seed=0)
    prefix = T.save_model(src, str(tmp_path / "model_1.ckpt"))
    ck = T.read_checkpoint(prefix)
    assert sorted(ck) == REFERENCE_NAMES
    assert ck["FC1/Variable"].shape == (1000, 100) and ck["Training/beta1_power"].shape == ()
    dst = _StubModel(1000, (100, 100), seed=1)
    T.restore_model(dst, prefix)
    assert dst.step == 2 and dst.b == src.b  # beta1_power = 0.9^(t+1)
    for a, b in ((src.p, dst.p), (src.m, dst.m), (src.v, dst.v), (src.ema, dst.ema)):
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_restore_matches_ema_by_suffix(tmp_path):
    """A checkpoint whose EMA slots carry another TF version's prefix still restores."""
    src = _StubModel(200, (30, 20), seed=3)
    t = T.model_tensors(src)
    t = {(k[len("bn/"):] if k.startswith("bn/BN") else k): v for k, v in t.items()}
    prefix = T.write_checkpoint(str(tmp_path / "alt.ckpt"), t)
    dst = _StubModel(200, (30, 20), seed=4)
    T.restore_model(dst, prefix)
    for k in src.ema:
        assert torch.equal(src.ema[k], dst.ema[k])
