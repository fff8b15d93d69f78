"""ctypes binding of libvptmcm.so (include/vptmcm.h).

Harness plumbing for bench.py and the pytest suite; the product's own host is
the JavaScript renderer over the N-API shim (js/, napi/). There is no CPU
fallback: if the HIP library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parents[2]
LIB_DIR = PKG / "lib"
# A/B and measurement builds (tools/variants.py): never beside the product library
VARIANT_DIR = PKG.parent / "build" / "variants"

OK, EINVAL, EHIP, ESTATE, ENOMEM, ECOMM = 0, -1, -2, -3, -4, -5
ALLREDUCE_INLINE = 1  # VPTMCM_ALLREDUCE_INLINE
ALLREDUCE_SHARDED = 2  # VPTMCM_ALLREDUCE_SHARDED
LAYOUT_LINEAR, LAYOUT_CORNER8, LAYOUT_BRICK8, LAYOUT_COLUMN4 = 0, 1, 2, 3
RENDERER_SPECTRAL, RENDERER_RGB = 0, 1
PHOTON_RGB_BYTES = 64
PHOTON_BYTES = 144
MAX_BINS = 12

# every symbol include/vptmcm.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "vptmcm_create", "vptmcm_destroy", "vptmcm_last_error", "vptmcm_set_volume",
    "vptmcm_volume_begin", "vptmcm_volume_write_block", "vptmcm_volume_end",
    "vptmcm_set_material_tf", "vptmcm_set_light", "vptmcm_set_spectrum", "vptmcm_set_params",
    "vptmcm_set_band", "vptmcm_comm_gather_bands",
    "vptmcm_reset", "vptmcm_render", "vptmcm_render_passes", "vptmcm_synchronize",
    "vptmcm_read_rgba16f", "vptmcm_read_rgb", "vptmcm_pack_radiance", "vptmcm_read_photons", "vptmcm_write_photons",
    "vptmcm_tonemap_artistic", "vptmcm_set_transfer_function", "vptmcm_set_environment",
    "vptmcm_enable_kernel_timing", "vptmcm_kernel_time", "vptmcm_comm_unique_id",
    "vptmcm_comm_init", "vptmcm_comm_allreduce_radiance", "vptmcm_comm_allreduce_radiance_ex",
    "vptmcm_comm_read_composite",
    "vptmcm_comm_barrier", "vptmcm_comm_allreduce_host", "vptmcm_debug_eval",
    "vptmcm_debug_verify", "vptmcm_debug_last_launch", "vptmcm_debug_schedule", "vptmcm_version",
    "vptmcm_read_composite", "vptmcm_composite", "vptmcm_group_devices", "vptmcm_set_macro_skip",
]
MAX_DEVICES = 8
GROUP_PEER, GROUP_RCCL = 0, 1


class Config(C.Structure):
    _fields_ = [("resolution", C.c_uint32), ("max_bins", C.c_uint32), ("device", C.c_int32),
                ("volume_layout", C.c_uint32), ("renderer", C.c_uint32),
                ("n_devices", C.c_uint32), ("devices", C.c_int32 * MAX_DEVICES),
                ("group_transport", C.c_uint32)]


class Params(C.Structure):
    _fields_ = [("extinction", C.c_float), ("anisotropy", C.c_float),
                ("max_bounces", C.c_uint32), ("steps", C.c_uint32), ("blur", C.c_float)]


class VptError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vptmcm error {code}: {msg}")
        self.code = code


_lib = None


def lib_path() -> Path:
    # VPTMCM_LIB=<name> selects build/variants/libvptmcm_<name>.so (outside the
    # shipped package): the cost-attribution builds (exp, exp_stamps; results
    # invalid) and tuning variants built by tools/variants.py for A/B sweeps
    # (tools only; never the product default)
    name = os.environ.get("VPTMCM_LIB", "")
    if name:
        if not name.replace("_", "").isalnum():
            raise ValueError(f"VPTMCM_LIB={name!r}: expected an alphanumeric variant name")
        return VARIANT_DIR / f"libvptmcm_{name}.so"
    return LIB_DIR / "libvptmcm.so"


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    if not p.exists():
        raise RuntimeError(f"{p} is not built: run `python __graft_entry__.py build` "
                           "(the HIP path has no fallback)")
    L = C.CDLL(str(p))
    vp, u8p, f32p, u32p = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_float), C.POINTER(C.c_uint32)
    sig = {
        "vptmcm_create": (C.c_int, [C.POINTER(Config), C.POINTER(vp)]),
        "vptmcm_destroy": (None, [vp]),
        "vptmcm_last_error": (C.c_char_p, [vp]),
        "vptmcm_set_volume": (C.c_int, [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32]),
        "vptmcm_volume_begin": (C.c_int, [vp, C.c_uint32, C.c_uint32, C.c_uint32]),
        "vptmcm_volume_write_block": (C.c_int, [vp, vp] + [C.c_uint32] * 6),
        "vptmcm_volume_end": (C.c_int, [vp]),
        "vptmcm_set_material_tf": (C.c_int, [vp, vp]),
        "vptmcm_set_light": (C.c_int, [vp, vp, f32p]),
        "vptmcm_set_spectrum": (C.c_int, [vp, f32p]),
        "vptmcm_set_params": (C.c_int, [vp, C.POINTER(Params)]),
        "vptmcm_set_band": (C.c_int, [vp, C.c_uint32, C.c_uint32]),
        "vptmcm_comm_gather_bands": (C.c_int, [vp, f32p]),
        "vptmcm_reset": (C.c_int, [vp, f32p, C.c_uint32]),
        # the per-pass calls take raw addresses (c_void_p): no ctypes pointer objects
        "vptmcm_render": (C.c_int, [vp, vp, C.c_uint32]),
        "vptmcm_render_passes": (C.c_int, [vp, vp, vp, C.c_uint32]),
        "vptmcm_synchronize": (C.c_int, [vp]),
        "vptmcm_read_rgba16f": (C.c_int, [vp, vp]),
        "vptmcm_read_rgb": (C.c_int, [vp, vp]),
        "vptmcm_pack_radiance": (C.c_int, [vp, vp]),
        "vptmcm_tonemap_artistic": (C.c_int, [vp, vp, vp]),
        "vptmcm_set_transfer_function": (C.c_int, [vp, vp, C.c_uint32, C.c_uint32]),
        "vptmcm_set_environment": (C.c_int, [vp, vp, C.c_uint32, C.c_uint32]),
        "vptmcm_read_photons": (C.c_int, [vp, vp]),
        "vptmcm_write_photons": (C.c_int, [vp, vp]),
        "vptmcm_enable_kernel_timing": (C.c_int, [vp, C.c_int]),
        "vptmcm_set_macro_skip": (C.c_int, [vp, C.c_int]),
        "vptmcm_kernel_time": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
        "vptmcm_comm_unique_id": (C.c_int, [u8p]),
        "vptmcm_comm_init": (C.c_int, [vp, u8p, C.c_int, C.c_int]),
        "vptmcm_comm_allreduce_radiance": (C.c_int, [vp]),
        "vptmcm_comm_allreduce_radiance_ex": (C.c_int, [vp, C.c_uint32]),
        "vptmcm_comm_read_composite": (C.c_int, [vp, f32p, f32p]),
        "vptmcm_comm_barrier": (C.c_int, [vp]),
        "vptmcm_comm_allreduce_host": (C.c_int, [vp, C.POINTER(C.c_double), C.c_int, C.c_int]),
        "vptmcm_debug_eval": (C.c_int, [vp, C.c_int, u32p, u32p, C.c_uint32]),
        "vptmcm_debug_verify": (C.c_int, [vp, C.c_int, C.c_uint32, C.c_uint64,
                                          C.POINTER(C.c_uint64), u32p, C.c_uint32]),
        "vptmcm_debug_last_launch": (C.c_int, [vp, u32p, C.POINTER(C.c_uint64)]),
        "vptmcm_debug_schedule": (C.c_int, [vp, u32p, C.c_uint32, u32p]),
        "vptmcm_version": (C.c_char_p, []),
        "vptmcm_read_composite": (C.c_int, [vp, vp, vp, vp]),
        "vptmcm_composite": (C.c_int, [vp]),
        "vptmcm_group_devices": (C.c_int, [vp, C.POINTER(C.c_int32), u32p]),
    }
    variant = bool(os.environ.get("VPTMCM_LIB"))
    for name, (res, args) in sig.items():
        if variant and not hasattr(L, name):
            continue  # an A/B variant built from an older revision lacks newer entry points
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _ptr(a: np.ndarray, ctype=C.c_void_p):
    return a.ctypes.data_as(ctype) if ctype is not C.c_void_p else C.c_void_p(a.ctypes.data)


def _f32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _u32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def mat_f32(mvp) -> np.ndarray:
    m = np.ascontiguousarray(mvp, dtype=np.float32).reshape(16)
    return m


class Renderer:
    """Thin handle wrapper (one HIP device, one stream)."""

    def __init__(self, resolution: int = 512, device: int = -1, layout: int = LAYOUT_CORNER8,
                 renderer: int = RENDERER_SPECTRAL, devices=None, transport: int = GROUP_PEER):
        """devices: a device list (vptmcm_config::n_devices): one handle, one
        photon-parallel replica per entry, composited on devices[0]."""
        self.L = load()
        cfg = Config(resolution, MAX_BINS, device, layout, renderer)
        if devices is not None:
            devices = list(devices)
            if not 1 <= len(devices) <= MAX_DEVICES:
                raise ValueError(f"1 to {MAX_DEVICES} devices, got {len(devices)}")
            cfg.n_devices = len(devices)
            for k, d in enumerate(devices):
                cfg.devices[k] = int(d)
            cfg.group_transport = int(transport)
        self.kind = renderer
        h = C.c_void_p()
        rc = self.L.vptmcm_create(C.byref(cfg), C.byref(h))
        if rc != OK:
            raise VptError(rc, self.L.vptmcm_last_error(None).decode())
        self.h = h
        self.R = resolution
        # Staging for the per-call hot-path arguments: numpy's .ctypes.data
        # costs ~2 us per array, so the matrix and the seeds are copied into
        # buffers whose addresses are taken once (the library copies both
        # during the call).
        self._m = np.zeros(16, np.float32)
        self._m_p = self._m.ctypes.data
        self._s = np.zeros(4096, np.uint32)
        self._s_p = self._s.ctypes.data

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "h", None):
            self.L.vptmcm_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc: int) -> None:
        if rc != OK:
            raise VptError(rc, self.L.vptmcm_last_error(self.h).decode())

    # -- inputs
    def set_volume(self, vol: np.ndarray) -> None:
        """vol: uint8 array [D, H, W] (x fastest)."""
        v = np.ascontiguousarray(vol, dtype=np.uint8)
        D, H, W = v.shape
        self._ck(self.L.vptmcm_set_volume(self.h, _ptr(v), W, H, D))

    def volume_begin(self, shape) -> None:
        """Start a block-wise ingest of a [D, H, W] volume (all zero until written)."""
        D, H, W = shape
        self._ck(self.L.vptmcm_volume_begin(self.h, W, H, D))

    def volume_write_block(self, origin, block) -> None:
        """One placement: uint8 [d, h, w] at origin (x, y, z)."""
        b = np.ascontiguousarray(block, dtype=np.uint8)
        d, hh, w = b.shape
        x, y, z = origin
        self._ck(self.L.vptmcm_volume_write_block(self.h, _ptr(b), x, y, z, w, hh, d))

    def volume_end(self) -> None:
        self._ck(self.L.vptmcm_volume_end(self.h))

    def volume_blocks(self, shape, blocks) -> None:
        """Block-wise ingest: blocks = iterable of (origin_xyz, uint8 [d,h,w])."""
        self.volume_begin(shape)
        for origin, b in blocks:
            self.volume_write_block(origin, b)
        self.volume_end()

    def set_material_tf(self, tf: np.ndarray) -> None:
        t = np.ascontiguousarray(tf, dtype=np.uint8)
        assert t.size == 256 * 256 * 4
        self._ck(self.L.vptmcm_set_material_tf(self.h, _ptr(t)))

    def set_light(self, spd: np.ndarray, direction) -> None:
        s = np.ascontiguousarray(spd, dtype=np.uint8)
        assert s.size == 256
        d = np.ascontiguousarray(direction, dtype=np.float32)
        self._ck(self.L.vptmcm_set_light(self.h, _ptr(s), _f32p(d)))

    def set_spectrum(self, buf: np.ndarray) -> None:
        b = np.zeros(64, np.float32)
        src = np.asarray(buf)
        if src.dtype == np.uint32:
            src = src.view(np.float32)
        b[: src.size] = src.astype(np.float32)
        self._ck(self.L.vptmcm_set_spectrum(self.h, _f32p(b)))

    def set_params(self, extinction=1.0, anisotropy=0.0, bounces=8, steps=8, blur=0.0) -> None:
        p = Params(extinction, anisotropy, bounces, steps, blur)
        self._ck(self.L.vptmcm_set_params(self.h, C.byref(p)))

    def set_band(self, y0: int, y1: int) -> None:
        """Mode B: reset/render only pixel rows [y0, y1) (multiples of 8)."""
        self._ck(self.L.vptmcm_set_band(self.h, int(y0), int(y1)))

    # -- hot path
    def reset(self, mvp, seed_bits: int) -> None:
        m = mat_f32(mvp)
        self._ck(self.L.vptmcm_reset(self.h, _f32p(m), int(seed_bits) & 0xFFFFFFFF))

    def _stage_matrix(self, mvp) -> int:
        # a scalar or a short array would broadcast below (len() is the cheap test)
        if (len(mvp) if hasattr(mvp, "__len__") else 0) != 16 and np.size(mvp) != 16:
            raise ValueError(f"matrix needs 16 values, got {np.size(mvp)}")
        try:
            self._m[:] = mvp  # 16 values (np.reshape alone costs ~1.7 us)
        except ValueError:
            self._m[:] = np.asarray(mvp, np.float32).ravel()  # e.g. a 4 x 4 matrix
        return self._m_p

    def render(self, mvp, seed_bits: int) -> None:
        rc = self.L.vptmcm_render(self.h, self._stage_matrix(mvp), int(seed_bits) & 0xFFFFFFFF)
        if rc != OK:
            self._ck(rc)

    def render_passes(self, mvp, seeds) -> None:
        n = len(seeds)
        if n <= self._s.size:
            self._s[:n] = seeds
            sp = self._s_p
        else:
            s = np.ascontiguousarray(seeds, dtype=np.uint32)
            sp = s.ctypes.data
        rc = self.L.vptmcm_render_passes(self.h, self._stage_matrix(mvp), sp, n)
        if rc != OK:
            self._ck(rc)

    def synchronize(self) -> None:
        self._ck(self.L.vptmcm_synchronize(self.h))

    def bind_render_passes(self, mvp, seeds):
        """A zero-argument callable that makes the render_passes(mvp, seeds)
        call, with the matrix and the seeds staged now into buffers of its own:
        a timed region then spends nothing on converting them (bench.py; the
        call itself is the C-ABI entry point, unchanged)."""
        m = np.array(self._m, copy=True)
        self._stage_matrix(mvp)
        m[:] = self._m
        s = np.array(seeds, dtype=np.uint32, copy=True)
        f, h, mp, sp, n, ck = self.L.vptmcm_render_passes, self.h, m.ctypes.data, s.ctypes.data, len(s), self._ck

        def call():
            rc = f(h, mp, sp, n)
            if rc != OK:
                ck(rc)
        call.buffers = (m, s)  # alive as long as the callable
        return call

    def bind_synchronize(self):
        """vptmcm_synchronize as a zero-argument callable (see bind_render_passes)."""
        f, h, ck = self.L.vptmcm_synchronize, self.h, self._ck

        def call():
            rc = f(h)
            if rc != OK:
                ck(rc)
        return call

    # -- outputs
    def read_rgba16f(self) -> np.ndarray:
        out = np.empty((self.R, self.R, 4), np.uint16)
        self._ck(self.L.vptmcm_read_rgba16f(self.h, _ptr(out)))
        return out

    def read_rgb(self) -> np.ndarray:
        """fp32 RGB of the last pass before the f16 store, [R, R, 3]."""
        out = np.empty((self.R, self.R, 3), np.float32)
        self._ck(self.L.vptmcm_read_rgb(self.h, _ptr(out)))
        return out

    def pack_radiance(self) -> np.ndarray:
        """(rgb*n, n) per pixel, [R, R, 4] float32 (what the composite all-reduces)."""
        out = np.empty((self.R, self.R, 4), np.float32)
        self._ck(self.L.vptmcm_pack_radiance(self.h, _ptr(out)))
        return out

    def tonemap_artistic(self, low=0.0, mid=0.5, high=1.0, saturation=1.0, gamma=2.2) -> np.ndarray:
        """WebGPUArtisticToneMapper on the current render target -> rgba8 [R, R, 4]."""
        p = np.array([low, mid, high, saturation, gamma], np.float32)
        out = np.zeros((self.R, self.R, 4), np.uint8)
        self._ck(self.L.vptmcm_tonemap_artistic(self.h, _ptr(p), _ptr(out)))
        return out

    def _photon_words(self) -> int:
        return (PHOTON_RGB_BYTES if self.kind == RENDERER_RGB else PHOTON_BYTES) // 4

    def set_transfer_function(self, rgba: np.ndarray) -> None:
        """RGB renderer: rgba8unorm-srgb TF image [H, W, 4] (setTransferFunction)."""
        t = np.ascontiguousarray(rgba, dtype=np.uint8)
        self._ck(self.L.vptmcm_set_transfer_function(self.h, _ptr(t), t.shape[1], t.shape[0]))

    def set_environment(self, rgba) -> None:
        """RGB renderer: the 1x1 environment texel (rgba8unorm)."""
        t = np.ascontiguousarray(np.asarray(rgba, dtype=np.uint8).reshape(4))
        self._ck(self.L.vptmcm_set_environment(self.h, _ptr(t), 1, 1))

    def read_photons(self) -> np.ndarray:
        """(R*R, words) uint32 in the reference's layout: 144-B PhotonSpectral
        (36 words) or, for the RGB renderer, 64-B Photon (16 words)."""
        out = np.empty((self.R * self.R, self._photon_words()), np.uint32)
        self._ck(self.L.vptmcm_read_photons(self.h, _ptr(out)))
        return out

    def write_photons(self, words: np.ndarray) -> None:
        w = np.ascontiguousarray(words, dtype=np.uint32)
        assert w.size == self.R * self.R * self._photon_words()
        self._ck(self.L.vptmcm_write_photons(self.h, _ptr(w)))

    # -- measurement
    def enable_kernel_timing(self, on: bool = True) -> None:
        self._ck(self.L.vptmcm_enable_kernel_timing(self.h, 1 if on else 0))

    def set_macro_skip(self, mode: str) -> None:
        """The macro-cell alpha bound: "off", "on" or "auto" (vptmcm_set_macro_skip)."""
        self._ck(self.L.vptmcm_set_macro_skip(self.h, {"off": 0, "on": 1, "auto": 2}[mode]))

    def kernel_time(self):
        ms, n = C.c_double(), C.c_uint64()
        self._ck(self.L.vptmcm_kernel_time(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    # -- multi-GPU
    def comm_init(self, uid: bytes, nranks: int, rank: int) -> None:
        u = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._ck(self.L.vptmcm_comm_init(self.h, u, nranks, rank))

    def allreduce_radiance(self, inline: bool = False, sharded: bool = False) -> None:
        """The cross-rank composite; inline=True runs it on the march stream
        (VPTMCM_ALLREDUCE_INLINE: soonest ready, the next march waits);
        sharded=True reduce-scatters instead (VPTMCM_ALLREDUCE_SHARDED: the
        next read_composite is collective, every rank calls it)."""
        flags = (ALLREDUCE_INLINE if inline else 0) | (ALLREDUCE_SHARDED if sharded else 0)
        if flags:
            self._ck(self.L.vptmcm_comm_allreduce_radiance_ex(self.h, flags))
        else:
            self._ck(self.L.vptmcm_comm_allreduce_radiance(self.h))

    def read_composite(self):
        rgb = np.empty((self.R, self.R, 3), np.float32)
        n = np.empty((self.R, self.R), np.float32)
        self._ck(self.L.vptmcm_comm_read_composite(self.h, _f32p(rgb), _f32p(n)))
        return rgb, n

    def read_composite_all(self):
        """vptmcm_read_composite: (rgba16f [R,R,4] u16, rgb [R,R,3] f32, counts [R,R] f32)."""
        q = np.empty((self.R, self.R, 4), np.uint16)
        rgb = np.empty((self.R, self.R, 3), np.float32)
        n = np.empty((self.R, self.R), np.float32)
        self._ck(self.L.vptmcm_read_composite(self.h, _ptr(q), _ptr(rgb), _ptr(n)))
        return q, rgb, n

    def composite(self) -> None:
        self._ck(self.L.vptmcm_composite(self.h))

    def group_devices(self) -> list:
        n = np.zeros(1, np.uint32)
        d = np.zeros(MAX_DEVICES, np.int32)
        self._ck(self.L.vptmcm_group_devices(self.h, d.ctypes.data_as(C.POINTER(C.c_int32)), _u32p(n)))
        return [int(x) for x in d[: int(n[0])]]

    def gather_bands(self) -> np.ndarray:
        """Mode B composite over the communicator: the fp32 image, bit-exact."""
        out = np.empty((self.R, self.R, 3), np.float32)
        self._ck(self.L.vptmcm_comm_gather_bands(self.h, _f32p(out)))
        return out

    def barrier(self) -> None:
        self._ck(self.L.vptmcm_comm_barrier(self.h))

    def allreduce_host(self, vals, op: str = "sum") -> np.ndarray:
        v = np.ascontiguousarray(vals, dtype=np.float64).copy()
        self._ck(self.L.vptmcm_comm_allreduce_host(
            self.h, v.ctypes.data_as(C.POINTER(C.c_double)), v.size, 1 if op == "max" else 0))
        return v

    # -- diagnostics
    def debug_eval(self, fn: int, inp: np.ndarray) -> np.ndarray:
        i = np.ascontiguousarray(inp, dtype=np.uint32)
        o = np.empty_like(i)
        self._ck(self.L.vptmcm_debug_eval(self.h, fn, _u32p(i), _u32p(o), i.size))
        return o


    def last_launch(self) -> dict:
        """What the last march launch ran (vptmcm_debug_last_launch)."""
        info = np.zeros(4, np.uint32)
        n = C.c_uint64()
        self._ck(self.L.vptmcm_debug_last_launch(self.h, _u32p(info), C.byref(n)))
        return {"mode": int(info[0]), "tpl": int(info[1]), "spec": bool(info[2] & 1),
                "macro": bool(info[2] & 2),
                "passes": int(info[3]), "launches": n.value}

    def debug_schedule(self) -> np.ndarray:
        """Per wave slot the packed tile of the last balanced-schedule march
        launch (tile | volume << 31, 0xffffffff idle; vptmcm_debug_schedule)."""
        n = np.zeros(1, np.uint32)
        self._ck(self.L.vptmcm_debug_schedule(self.h, None, 0, _u32p(n)))
        out = np.empty(int(n[0]), np.uint32)
        self._ck(self.L.vptmcm_debug_schedule(self.h, _u32p(out), out.size, _u32p(n)))
        return out

    def uniform_bins(self) -> bool:
        """True when the current spectrum takes the arithmetic bin search."""
        return self.debug_verify(14, 0, 1, 0)[0] == 0

    def debug_verify(self, fn: int, lo: int = 0, count: int = 1 << 32, nfirst: int = 16):
        bad = C.c_uint64()
        first = np.zeros(max(nfirst, 1), np.uint32)
        self._ck(self.L.vptmcm_debug_verify(self.h, fn, lo, count, C.byref(bad), _u32p(first),
                                            nfirst))
        return bad.value, first[: min(nfirst, bad.value)]


def unique_id() -> bytes:
    L = load()
    buf = (C.c_uint8 * 128)()
    rc = L.vptmcm_comm_unique_id(buf)
    if rc != OK:
        raise VptError(rc, L.vptmcm_last_error(None).decode())
    return bytes(buf)
