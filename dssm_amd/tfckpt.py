"""TF1.x ``tf.train.Saver`` checkpoints (new_dssm.py:248 ``saver = tf.train.Saver()``, :331
``saver.save(sess, "model/model_1.ckpt")``) written and read without TensorFlow.

A V2 checkpoint ``<prefix>`` is three files:

* ``<prefix>.data-00000-of-00001``: every tensor's little-endian bytes, back to back;
* ``<prefix>.index``: a LevelDB-format table (sorted keys, prefix-compressed entries with restart
  points, blocks closed by a type byte and a masked CRC-32C, an index block of block handles and a
  48-byte footer ending in magic 0xdb4775248b80fb57).  Key "" holds a ``BundleHeaderProto``
  {num_shards: 1, version {producer: 1}}; every tensor name holds a ``BundleEntryProto``
  {dtype, shape, offset, size, crc32c = masked CRC-32C of its bytes};
* ``checkpoint`` in the same directory: the text proto naming the latest prefix.

``tf.train.Saver.save`` also writes a ``.meta`` graph (MetaGraphDef); ``api.Saver.save`` writes its
own ``.meta`` instead (a JSON description of the api's DSSMGraph that ``api.import_meta_graph``
rebuilds the graph from), since the graph here is not a TF graph.  The protobuf messages of the
bundle are encoded by hand (a handful of fields).

Variable names follow TF1.x's naming of the reference graph (new_dssm.py:117-217, with
``batch_normalization`` :62-88): ``tf.Variable`` takes the enclosing name scope, a second
``variable_scope('bn')`` in the same name scope opens ``bn_1``, ExponentialMovingAverage shadows
of the ``tf.nn.moments`` outputs are slots named ``<op name>/ExponentialMovingAverage`` under the
enclosing variable scope ``bn``, Adam slots are ``<var>/Adam`` (m) and ``<var>/Adam_1`` (v), and
the beta powers are created under the ``Training`` name scope:

=====================  =====================================================================
dssm_amd               TF1.x variable
=====================  =====================================================================
W{l}, b{l}             FC{l}/Variable, FC{l}/Variable_1
bn{l}_q_beta / gamma   BN{l}/bn/beta, BN{l}/bn/gamma        (doc tower: BN{l}/bn_1/...)
bn{l}_q_mean / var     bn/BN{l}/bn/moments/Squeeze[_1]/ExponentialMovingAverage (doc: bn_1)
Adam m / v of X        X/Adam, X/Adam_1
beta powers            Training/beta1_power, Training/beta2_power
=====================  =====================================================================

Layers past the reference's two (C2's FC3 / BN3) continue the pattern.  TensorFlow is not in this
image, so these names and the file layout are pinned by the format's specification and by the
round trips and golden bytes of tests/test_tfckpt.py, not by a TF reader (parity unpinned).
``read_checkpoint`` accepts any V2 bundle of float32 / int64 tensors (multi-block indexes, TF's
prefix compression), and ``restore`` also matches EMA shadows by their ``.../moments/Squeeze[_1]
/ExponentialMovingAverage`` suffix, since that slot's prefix depends on the TF version.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from typing import Dict, List, Tuple

import numpy as np

MAGIC = 0xDB4775248B80FB57
DT_FLOAT, DT_INT64 = 1, 9
_DTYPES = {DT_FLOAT: np.float32, DT_INT64: np.int64}
_CODES = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.int64): DT_INT64}


def crc32c(data, crc: int = 0) -> int:
    from . import _lib
    buf = np.ascontiguousarray(np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray))
                               else data)
    return int(_lib.load().dssm_crc32c(crc, buf.ctypes.data_as(C.c_void_p), buf.nbytes))


def mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask(m: int) -> int:
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---- protobuf / varint helpers --------------------------------------------------------------
def _varint(x: int) -> bytes:
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        if not c & 0x80:
            return x, i
        s += 7


def _field(num: int, wire: int) -> bytes:
    return _varint(num << 3 | wire)


def _len_field(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def _parse_fields(b: bytes) -> List[Tuple[int, int, object]]:
    out, i = [], 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wire = key >> 3, key & 7
        if wire == 0:
            v, i = _read_varint(b, i)
        elif wire == 1:
            v, i = struct.unpack_from("<Q", b, i)[0], i + 8
        elif wire == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        elif wire == 5:
            v, i = struct.unpack_from("<I", b, i)[0], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wire}")
        out.append((num, wire, v))
    return out


def _header_proto() -> bytes:
    # BundleHeaderProto {num_shards = 1; endianness = LITTLE (default); version {producer = 1}}
    return _field(1, 0) + _varint(1) + _len_field(3, _field(1, 0) + _varint(1))


def _entry_proto(dtype: int, shape, offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_len_field(2, _field(1, 0) + _varint(int(d))) for d in shape)
    out = _field(1, 0) + _varint(dtype) + _len_field(2, dims)
    if offset:
        out += _field(4, 0) + _varint(offset)
    if size:
        out += _field(5, 0) + _varint(size)
    return out + _field(6, 5) + struct.pack("<I", crc)


def _parse_entry(b: bytes) -> dict:
    e = {"dtype": DT_FLOAT, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None}
    for num, _w, v in _parse_fields(b):
        if num == 1:
            e["dtype"] = v
        elif num == 2:
            for dn, _dw, dv in _parse_fields(v):
                if dn == 2:
                    size = dict((f[0], f[2]) for f in _parse_fields(dv)).get(1, 0)
                    e["shape"].append(size - (1 << 64) if size >= 1 << 63 else size)
        elif num == 3:
            e["shard_id"] = v
        elif num == 4:
            e["offset"] = v
        elif num == 5:
            e["size"] = v
        elif num == 6:
            e["crc32c"] = v
        elif num == 7:
            raise ValueError("partitioned (sliced) tensors are not supported")
    return e


# ---- LevelDB table ---------------------------------------------------------------------------
def _block(entries: List[Tuple[bytes, bytes]], restart_interval: int) -> bytes:
    out, restarts, prev = bytearray(), [], b""
    for k, (key, val) in enumerate(entries):
        shared = 0
        if k % restart_interval == 0:
            restarts.append(len(out))
        else:
            while shared < min(len(prev), len(key)) and prev[shared] == key[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(key) - shared) + _varint(len(val)) + key[shared:] + val
        prev = key
    if not restarts:
        restarts = [0]
    out += b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))
    return bytes(out)


def _block_with_trailer(contents: bytes) -> bytes:
    trailer_type = b"\x00"  # kNoCompression
    return contents + trailer_type + struct.pack("<I", mask(crc32c(contents + trailer_type)))


def _handle(offset: int, size: int) -> bytes:
    return _varint(offset) + _varint(size)


def write_table(items: Dict[bytes, bytes], block_bytes: int = 4096) -> bytes:
    """LevelDB-format table of sorted (key, value) items (TF's table_builder layout)."""
    keys = sorted(items)
    out, index = bytearray(), []
    blk: List[Tuple[bytes, bytes]] = []
    size = 0

    def flush():
        nonlocal blk, size
        if not blk:
            return
        contents = _block(blk, 16)
        index.append((blk[-1][0], _handle(len(out), len(contents))))
        out.extend(_block_with_trailer(contents))
        blk, size = [], 0

    for k in keys:
        blk.append((k, items[k]))
        size += len(k) + len(items[k]) + 8
        if size >= block_bytes:
            flush()
    flush()
    meta = _block([], 16)
    meta_h = _handle(len(out), len(meta))
    out.extend(_block_with_trailer(meta))
    idx = _block(index, 1)
    idx_h = _handle(len(out), len(idx))
    out.extend(_block_with_trailer(idx))
    footer = (meta_h + idx_h).ljust(40, b"\x00") + struct.pack("<Q", MAGIC)
    return bytes(out + footer)


def _read_block(buf: bytes, offset: int, size: int) -> List[Tuple[bytes, bytes]]:
    contents = buf[offset:offset + size]
    ttype, crc = buf[offset + size], struct.unpack_from("<I", buf, offset + size + 1)[0]
    if ttype != 0:
        raise ValueError("compressed index blocks are not supported")
    if unmask(crc) != crc32c(buf[offset:offset + size + 1]):
        raise ValueError("index block checksum mismatch")
    nrest = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    end = len(contents) - 4 - 4 * nrest
    out, i, prev = [], 0, b""
    while i < end:
        shared, i = _read_varint(contents, i)
        nonshared, i = _read_varint(contents, i)
        vlen, i = _read_varint(contents, i)
        key = prev[:shared] + contents[i:i + nonshared]
        i += nonshared
        out.append((key, contents[i:i + vlen]))
        i += vlen
        prev = key
    return out


def read_table(buf: bytes) -> Dict[bytes, bytes]:
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != MAGIC:
        raise ValueError("not a table file (bad magic)")
    f = buf[len(buf) - 48:]
    _mo, i = _read_varint(f, 0)
    _ms, i = _read_varint(f, i)
    io, i = _read_varint(f, i)
    isz, i = _read_varint(f, i)
    items: Dict[bytes, bytes] = {}
    for _k, h in _read_block(buf, io, isz):
        o, j = _read_varint(h, 0)
        s, _ = _read_varint(h, j)
        items.update(_read_block(buf, o, s))
    return items


# ---- bundles ---------------------------------------------------------------------------------
def write_checkpoint(prefix: str, tensors: Dict[str, np.ndarray]) -> str:
    """Write a V2 bundle (``prefix``.index / .data-00000-of-00001) and the directory's
    ``checkpoint`` file; returns ``prefix`` (what Saver.save returns)."""
    d = os.path.dirname(os.path.abspath(prefix))
    os.makedirs(d, exist_ok=True)
    items = {b"": _header_proto()}
    offset = 0
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name])
            if not a.flags.c_contiguous:
                a = a.copy()  # (np.ascontiguousarray would turn a scalar into shape (1,))
            if a.dtype not in _CODES:
                raise TypeError(f"{name}: dtype {a.dtype} (float32 / int64 only)")
            raw = a.astype(a.dtype.newbyteorder("<"), copy=False)
            f.write(raw.tobytes())
            items[name.encode()] = _entry_proto(_CODES[a.dtype], a.shape, offset, a.nbytes,
                                                mask(crc32c(raw.reshape(-1).view(np.uint8))))
            offset += a.nbytes
    with open(prefix + ".index", "wb") as f:
        f.write(write_table(items))
    base = os.path.basename(prefix)
    with open(os.path.join(d, "checkpoint"), "w") as f:
        f.write(f'model_checkpoint_path: "{base}"\nall_model_checkpoint_paths: "{base}"\n')
    return prefix


def read_checkpoint(prefix: str) -> Dict[str, np.ndarray]:
    with open(prefix + ".index", "rb") as f:
        items = read_table(f.read())
    hdr = dict((n, v) for n, _w, v in _parse_fields(items.pop(b"", b"")))
    nshards = hdr.get(1, 1)
    if hdr.get(2, 0) != 0:
        raise ValueError("big-endian checkpoints are not supported")
    out: Dict[str, np.ndarray] = {}
    data = {}
    for key, val in items.items():
        e = _parse_entry(val)
        if e["dtype"] not in _DTYPES:
            raise TypeError(f"{key.decode()}: unsupported dtype {e['dtype']}")
        sh = e["shard_id"]
        if sh not in data:
            data[sh] = np.memmap(f"{prefix}.data-{sh:05d}-of-{nshards:05d}", np.uint8, mode="r")
        raw = np.asarray(data[sh][e["offset"]:e["offset"] + e["size"]])
        if e["crc32c"] is not None and unmask(e["crc32c"]) != crc32c(raw):
            raise ValueError(f"{key.decode()}: data checksum mismatch")
        out[key.decode()] = raw.view(_DTYPES[e["dtype"]]).reshape(e["shape"]).copy()
    return out


def latest_checkpoint(directory: str):
    """tf.train.latest_checkpoint: the prefix the directory's ``checkpoint`` file names."""
    p = os.path.join(directory, "checkpoint")
    if not os.path.exists(p):
        return None
    for line in open(p):
        if line.startswith("model_checkpoint_path:"):
            name = line.split(":", 1)[1].strip().strip('"')
            return name if os.path.isabs(name) else os.path.join(directory, name)
    return None


# ---- the reference graph's variable names -----------------------------------------------------
def variable_names(n_layers: int) -> Dict[str, str]:
    """dssm_amd parameter / EMA key -> TF1.x variable name (module doc table)."""
    out = {}
    for l in range(1, n_layers + 1):
        out[f"W{l}"] = f"FC{l}/Variable"
        out[f"b{l}"] = f"FC{l}/Variable_1"
        for t, sc in (("q", "bn"), ("d", "bn_1")):
            out[f"bn{l}_{t}_beta"] = f"BN{l}/{sc}/beta"
            out[f"bn{l}_{t}_gamma"] = f"BN{l}/{sc}/gamma"
            out[f"bn{l}_{t}_mean"] = f"bn/BN{l}/{sc}/moments/Squeeze/ExponentialMovingAverage"
            out[f"bn{l}_{t}_var"] = f"bn/BN{l}/{sc}/moments/Squeeze_1/ExponentialMovingAverage"
    return out


BETA_POWERS = ("Training/beta1_power", "Training/beta2_power")


def model_tensors(model) -> Dict[str, np.ndarray]:
    """Every variable tf.train.Saver() saves for the reference graph, from a DSSM model."""
    names = variable_names(len(model.widths))
    out = {}
    m, v = model.named_adam()
    for k, t in model.named_params().items():
        out[names[k]] = t.detach().cpu().numpy().astype(np.float32)
        out[names[k] + "/Adam"] = m[k].detach().cpu().numpy().astype(np.float32)
        out[names[k] + "/Adam_1"] = v[k].detach().cpu().numpy().astype(np.float32)
    for k, t in model.named_ema().items():
        out[names[k]] = t.detach().cpu().numpy().astype(np.float32)
    b1, b2 = model.beta_powers()
    out[BETA_POWERS[0]] = np.array(b1, np.float32)
    out[BETA_POWERS[1]] = np.array(b2, np.float32)
    return out


def _lookup(ck: Dict[str, np.ndarray], name: str) -> np.ndarray:
    if name in ck:
        return ck[name]
    if "/moments/" in name:  # EMA slot prefixes vary across TF versions: match the suffix
        tail = name.split("/", 1)[1]
        hits = [k for k in ck if k.endswith(tail)]
        if len(hits) == 1:
            return ck[hits[0]]
    raise KeyError(f"checkpoint has no variable {name}")


def restore_model(model, prefix: str):
    """Load a checkpoint written by ``save_model`` (or by TF for the same graph) into ``model``."""
    ck = read_checkpoint(prefix)
    names = variable_names(len(model.widths))
    pv = model.named_params()
    params = {k: _lookup(ck, names[k]).reshape(pv[k].shape) for k in pv}
    ema = {k: _lookup(ck, names[k]) for k in model.named_ema()}
    m = {k: _lookup(ck, names[k] + "/Adam") for k in pv}
    v = {k: _lookup(ck, names[k] + "/Adam_1") for k in pv}
    b1, b2 = (float(_lookup(ck, n)) for n in BETA_POWERS)
    # TF keeps no step counter: beta1_power starts at beta1 and gains a factor per step
    beta1 = float(getattr(model, "beta1", 0.9))
    step = max(0, int(round(np.log(b1) / np.log(beta1))) - 1) if 0 < b1 < 1 and 0 < beta1 < 1 else 0
    model.load_adam_state(m, v, b1, b2, step)
    model.load_params(params, ema=ema)


def save_model(model, prefix: str) -> str:
    return write_checkpoint(prefix, model_tensors(model))
