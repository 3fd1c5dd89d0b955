"""C-ABI checks that need no GPU: libdssm.so loads, exports every function include/dssm.h
declares, and its host-side layout/sizing functions agree with the reference's parameter set."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dssm.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dssm_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from dssm_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from dssm_amd.build import build
        build()
    return _lib.load()


def test_exports_every_declared_function(lib):
    from dssm_amd import _lib
    declared = header_functions()
    assert len(declared) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (dssm_\w+)", out))
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    # and the ctypes binding covers all of them
    assert set(declared) <= set(_lib.exported_symbols()), set(declared) - set(_lib.exported_symbols())


def cfg(lib, D=30000, widths=(300, 300, 128), BS=1024, NEG=4, dtype=1, nnz=None):
    from dssm_amd import _lib
    c = _lib.dssm_config()
    c.abi_version = _lib.DSSM_ABI_VERSION
    c.trigram_d, c.n_layers = D, len(widths)
    for i, w in enumerate(widths):
        c.widths[i] = w
    c.query_bs, c.neg = BS, NEG
    c.max_nnz = nnz if nnz is not None else BS * (2 + NEG) * 96
    c.compute_dtype = dtype
    c.gamma, c.bn_eps, c.ema_decay, c.lr, c.beta1, c.beta2, c.adam_eps = 20, 1e-3, .5, .01, .9, .999, 1e-8
    return c


def test_layout_matches_reference_variables(lib):
    from dssm_amd import _lib
    c = cfg(lib)
    assert lib.dssm_config_check(C.byref(c)) == 0
    n = lib.dssm_param_layout(C.byref(c), None, 0)
    segs = (_lib.dssm_segment * n)()
    lib.dssm_param_layout(C.byref(c), segs, n)
    names = [s.name.decode() for s in segs]
    assert names[:3] == ["fc1", "fc2", "fc3"]
    real = sum(s.rows * s.cols for s in segs)
    assert real == 9_132_040  # trainable parameters at C2
    offs = [(s.offset, s.offset + s.rows * s.cols) for s in segs]
    for (a0, a1), (b0, b1) in zip(offs, offs[1:]):
        assert a1 <= b0 and b0 % 64 == 0
    assert lib.dssm_param_count(C.byref(c)) >= offs[-1][1]
    assert lib.dssm_ema_count(C.byref(c)) == 4 * (300 + 300 + 128)
    assert lib.dssm_workspace_bytes(C.byref(c)) > 0


@pytest.mark.parametrize("bad", [dict(widths=(300, 301)), dict(NEG=0), dict(NEG=16), dict(BS=0),
                                 dict(widths=(300, 1024)), dict(dtype=7)])
def test_config_rejects_invalid(lib, bad):
    c = cfg(lib, **bad)
    assert lib.dssm_config_check(C.byref(c)) < 0
    assert lib.dssm_last_error()


def test_missing_library_fails_loudly(tmp_path):
    from dssm_amd import _lib
    saved = _lib._lib
    try:
        _lib._lib = None
        with pytest.raises(_lib.DssmError):
            _lib.load(str(tmp_path / "nope.so"))
    finally:
        _lib._lib = saved
