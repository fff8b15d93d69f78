"""The C-ABI library loads and exports every symbol include/vptmcm.h declares
(no compute calls: this container has no GPU)."""
import ctypes as C
import re
from pathlib import Path

import pytest

import vptmcm

HEADER = Path(__file__).resolve().parents[1] / "include" / "vptmcm.h"


def declared_symbols():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(vptmcm_\w+)\(", text, re.M)))


def test_header_and_binding_agree():
    assert sorted(vptmcm.EXPORTS) == declared_symbols()


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(str(vptmcm.lib_path()))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_argument_errors():
    L = vptmcm.load()
    assert b"gfx950" in L.vptmcm_version()
    # invalid configs are rejected before any device call
    cfg = vptmcm._lib.Config(0, 12, -1, 0)
    h = C.c_void_p()
    assert L.vptmcm_create(C.byref(cfg), C.byref(h)) == vptmcm._lib.EINVAL
    assert b"resolution" in L.vptmcm_last_error(None)
    cfg = vptmcm._lib.Config(64, 11, -1, 0)
    assert L.vptmcm_create(C.byref(cfg), C.byref(h)) == vptmcm._lib.EINVAL
    assert b"max_bins" in L.vptmcm_last_error(None)
    assert L.vptmcm_set_params(None, None) == vptmcm._lib.EINVAL


def test_no_silent_cpu_fallback(monkeypatch, tmp_path):
    """The product fails loudly when the HIP library is absent."""
    monkeypatch.setattr(vptmcm._lib, "_lib", None)
    monkeypatch.setattr(vptmcm._lib, "LIB_DIR", tmp_path)
    with pytest.raises(RuntimeError, match="not built"):
        vptmcm._lib.load()


def test_hot_path_argument_staging():
    """Renderer stages the matrix and the seeds in buffers whose addresses are
    taken once; every accepted matrix form lands as the same 16 floats
    (row-major flattening of a 4 x 4, as np.reshape would give)."""
    import numpy as np
    from vptmcm import configs as cf

    r = vptmcm.Renderer.__new__(vptmcm.Renderer)  # no device: staging only
    r._m = np.zeros(16, np.float32)
    r._m_p = r._m.ctypes.data
    m = cf.default_mvp_inverse()
    for form in (m, m.reshape(4, 4), [float(v) for v in m], m.astype(np.float64)):
        assert r._stage_matrix(form) == r._m_p
        assert np.array_equal(r._m.view(np.uint32), m.view(np.uint32))
    # a scalar or a short array must not broadcast into all 16 entries
    for bad in (1.0, np.ones(1, np.float32), np.ones(4, np.float32), np.ones((4, 1), np.float32),
                [1.0] * 15):
        with pytest.raises(ValueError, match="16 values"):
            r._stage_matrix(bad)
