"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; the product never imports it.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
PHOTON_WORDS = 36


class Uniforms(C.Structure):  # orc_uniforms (render UBO, wgsl:8-18)
    _fields_ = [("mvp_inverse", C.c_float * 16), ("inv_res", C.c_float * 2),
                ("seed_bits", C.c_uint32), ("blur", C.c_float), ("extinction", C.c_float),
                ("anisotropy", C.c_float), ("max_bounces", C.c_uint32), ("steps", C.c_uint32),
                ("light_dir", C.c_float * 3)]


_L = None
_L_ALT = None


def load(alt: bool = False) -> C.CDLL:
    """liboracle.so (the arithmetic specification) or, with alt=True,
    liboracle_alt.so (libm transcendentals, true division, no fused products:
    the statistical parity test's alternative legal WGSL arithmetic)."""
    global _L, _L_ALT
    if alt:
        if _L_ALT is None:
            _L_ALT = _bind(HERE / "liboracle_alt.so")
        return _L_ALT
    if _L is None:
        _L = _bind(HERE / "liboracle.so")
    return _L


def _bind(p: Path) -> C.CDLL:
    if not p.exists():
        raise RuntimeError(f"{p} not built (make -C oracle)")
    L = C.CDLL(str(p))
    vp = C.c_void_p
    L.orc_reset.argtypes = [C.c_uint32, C.POINTER(Uniforms), vp, vp, C.c_int]
    L.orc_reset.restype = None
    L.orc_render.argtypes = [C.c_uint32, C.POINTER(Uniforms), vp, vp, C.c_uint32, C.c_uint32,
                             C.c_uint32, vp, vp, vp, vp, vp, C.c_int, C.c_uint32, C.c_uint32]
    L.orc_render.restype = None
    L.orc_hash.argtypes = [C.c_uint32]
    L.orc_hash.restype = C.c_uint32
    L.orc_hash3.argtypes = [C.c_uint32] * 3
    L.orc_hash3.restype = C.c_uint32
    for f in ("orc_log", "orc_sin", "orc_cos"):
        getattr(L, f).argtypes = [C.c_float]
        getattr(L, f).restype = C.c_float
    L.orc_f2h.argtypes = [C.c_float]
    L.orc_f2h.restype = C.c_uint16
    L.orc_sample_volume.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.POINTER(C.c_float)]
    L.orc_sample_volume.restype = C.c_float
    L.orc_sample_tf.argtypes = [vp, C.c_float, C.c_float, C.POINTER(C.c_float)]
    L.orc_sample_tf.restype = None
    L.orc_sample_light.argtypes = [vp, C.c_float]
    L.orc_sample_light.restype = C.c_float
    L.orc_reset_rgb.argtypes = [C.c_uint32, C.POINTER(Uniforms), vp, C.c_int]
    L.orc_reset_rgb.restype = None
    L.orc_render_rgb.argtypes = [C.c_uint32, C.POINTER(Uniforms), vp, C.c_uint32, C.c_uint32,
                                 C.c_uint32, vp, C.c_uint32, C.c_uint32, vp, vp, vp, C.c_int]
    L.orc_render_rgb.restype = None
    L.orc_srgb_to_linear.argtypes = [C.c_uint8]
    L.orc_srgb_to_linear.restype = C.c_float
    L.orc_tonemap_artistic.argtypes = [vp, C.c_uint32, vp, vp]
    L.orc_tonemap_artistic.restype = None
    L.orc_eval_batch.argtypes = [C.c_int, vp, vp, C.c_uint32]
    L.orc_eval_batch.restype = None
    return L


def _vp(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None else None


class Oracle:
    """Stateful mirror of one renderer: photon buffer + inputs, CPU only."""

    def __init__(self, R: int, alt: bool = False):
        self.L = load(alt)
        self.R = R
        self.photons = np.zeros((R * R, PHOTON_WORDS), np.uint32)
        self.spectrum = np.zeros(64, np.float32)
        self.volume = None
        self.tf = np.zeros((256, 256, 4), np.uint8)
        self.light = np.zeros(256, np.uint8)
        self.light_dir = np.array([1, 0, 0], np.float32)
        self.params = dict(extinction=1.0, anisotropy=0.0, bounces=8, steps=8, blur=0.0)

    def uniforms(self, mvp, seed_bits: int) -> Uniforms:
        u = Uniforms()
        u.mvp_inverse[:] = [float(x) for x in np.asarray(mvp, np.float32).reshape(16)]
        inv = float(np.float32(1.0 / self.R))
        u.inv_res[:] = [inv, inv]
        u.seed_bits = int(seed_bits) & 0xFFFFFFFF
        u.blur = self.params["blur"]
        u.extinction = self.params["extinction"]
        u.anisotropy = self.params["anisotropy"]
        u.max_bounces = self.params["bounces"]
        u.steps = self.params["steps"]
        u.light_dir[:] = [float(x) for x in self.light_dir]
        return u

    def set_spectrum(self, buf) -> None:
        b = np.zeros(64, np.float32)
        src = np.asarray(buf)
        if src.dtype == np.uint32:
            src = src.view(np.float32)
        b[: src.size] = src
        self.spectrum = b

    def reset(self, mvp, seed_bits: int, nthreads: int = 8) -> None:
        u = self.uniforms(mvp, seed_bits)
        self.L.orc_reset(self.R, C.byref(u), _vp(self.spectrum), _vp(self.photons), nthreads)

    def render(self, mvp, seed_bits: int, nthreads: int = 8, rows=None):
        """One pass; returns (rgb32 [R,R,3], rgba16 [R,R,4])."""
        v = np.ascontiguousarray(self.volume, dtype=np.uint8)
        D, H, W = v.shape
        u = self.uniforms(mvp, seed_bits)
        rgb = np.zeros((self.R, self.R, 3), np.float32)
        rgba = np.zeros((self.R, self.R, 4), np.uint16)
        y0, y1 = rows if rows else (0, 0)
        tf = np.ascontiguousarray(self.tf, dtype=np.uint8)
        light = np.ascontiguousarray(self.light, dtype=np.uint8)
        self.L.orc_render(self.R, C.byref(u), _vp(self.spectrum), _vp(v), W, H, D, _vp(tf),
                          _vp(light), _vp(self.photons), _vp(rgb), _vp(rgba), nthreads, y0, y1)
        return rgb, rgba

    def tonemap_artistic(self, rgba16: np.ndarray, low=0.0, mid=0.5, high=1.0, saturation=1.0,
                         gamma=2.2) -> np.ndarray:
        """ArtisticToneMapper.wgsl on an rgba16f image, double precision -> rgba8."""
        src = np.ascontiguousarray(rgba16, dtype=np.uint16)
        out = np.zeros(src.shape[:-1] + (4,), np.uint8)
        p = np.array([low, mid, high, saturation, gamma], np.float32)
        self.L.orc_tonemap_artistic(_vp(src), src.size // 4, _vp(p), _vp(out))
        return out

    # primitives
    def eval_batch(self, fn: int, inp: np.ndarray) -> np.ndarray:
        i = np.ascontiguousarray(inp, dtype=np.uint32)
        o = np.empty_like(i)
        self.L.orc_eval_batch(fn, _vp(i), _vp(o), i.size)
        return o


class OracleRGB(Oracle):
    """The RGB sibling renderer ('mcm-compute', MCMComputeRenderer.wgsl): 64-B
    photons, an rgba8unorm-srgb TF image [H, W, 4] and a 1x1 environment texel."""
    PHOTON_WORDS_RGB = 16

    def __init__(self, R: int):
        super().__init__(R)
        self.photons = np.zeros((R * R, self.PHOTON_WORDS_RGB), np.uint32)
        self.tf = np.array([[[255, 0, 0, 0], [255, 0, 0, 255]]], np.uint8)  # the ctor's 2x1 default
        self.env = np.array([255, 255, 255, 255], np.uint8)

    def reset(self, mvp, seed_bits: int, nthreads: int = 8) -> None:
        u = self.uniforms(mvp, seed_bits)
        self.L.orc_reset_rgb(self.R, C.byref(u), _vp(self.photons), nthreads)

    def render(self, mvp, seed_bits: int, nthreads: int = 8, rows=None):
        """One pass; returns (None, rgba16 [R,R,4])."""
        v = np.ascontiguousarray(self.volume, dtype=np.uint8)
        D, H, W = v.shape
        u = self.uniforms(mvp, seed_bits)
        rgba = np.zeros((self.R, self.R, 4), np.uint16)
        tf = np.ascontiguousarray(self.tf, dtype=np.uint8)
        env = np.ascontiguousarray(self.env, dtype=np.uint8)
        self.L.orc_render_rgb(self.R, C.byref(u), _vp(v), W, H, D, _vp(tf), tf.shape[1], tf.shape[0],
                              _vp(env), _vp(self.photons), _vp(rgba), nthreads)
        return None, rgba
