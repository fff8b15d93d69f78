"""Synthetic inputs of BASELINE.md's configs (C1-C5) and the seed streams.

The reference's renderer reads its inputs from the DOM/UI; the benchmark and
parity tests synthesise the same formats:
  volume   uint8 [D, H, W], x fastest          (WebGPUVolume.js:55-93)
  TF       uint8 [256 rows=density, 256 cols=wavelength, 4]
                                               (MaterialTransferFunction.js:22,56-75)
  light    uint8 [256] SPD + direction          (js:82-83 defaults: 100s, [1,0,0])
  spectrum f32 [64] packed buffer               (js:311-312)
"""
from __future__ import annotations

import ctypes as C
import json
import os
from pathlib import Path

import numpy as np

from ._lib import LIB_DIR

REPO = Path(__file__).resolve().parents[3]
GOLDEN = REPO / "tests" / "golden"

# invert(P*V*M) for the default camera (WebGPURenderingContext.js:37-39:
# translation [0,0,2], fovy 1, aspect 1, near .1, far 100; model = translate(-.5)),
# as computed by the reference's gl-matrix (tests/golden/mvp_inverse.json "default";
# equality is asserted by tests/test_configs.py).
DEFAULT_MVP_INVERSE_BITS = np.array(
    [0x3F0BDA7B, 0x80000000, 0x80000000, 0x80000000, 0x80000000, 0x3F0BDA7B, 0x80000000,
     0x80000000, 0xC01FD70A, 0xC01FD70A, 0xC147CCCD, 0xC09FD70A, 0x402028F6, 0x402028F6,
     0x41383333, 0x40A028F6], dtype=np.uint32)


def default_mvp_inverse() -> np.ndarray:
    return DEFAULT_MVP_INVERSE_BITS.view(np.float32).copy()


def golden_mvp(name: str) -> np.ndarray:
    d = json.loads((GOLDEN / "mvp_inverse.json").read_text())
    return np.array(d["cameras"][name]["bits"], dtype=np.uint32).view(np.float32)


def spectrum_buffer(layout: str = "12") -> np.ndarray:
    """The 64-f32 buffer the reference uploads for a bin layout (golden fixture
    produced by the reference's compute_spectral_coefficients)."""
    d = json.loads((GOLDEN / "spectrum_buffers.json").read_text())
    return np.array(d["layouts"][layout]["buffer_bits"], dtype=np.uint32).view(np.float32)


# ----------------------------------------------------------------- seeds
def pcg(v: int) -> int:
    x = (v * 747796405 + 2891336453) & 0xFFFFFFFF
    x = (((x >> ((x >> 28) + 4)) ^ x) * 277803737) & 0xFFFFFFFF
    return ((x >> 22) ^ x) & 0xFFFFFFFF


def seed_bits(k: int, rank: int = 0) -> int:
    """Seed bits of pass k (k = 0 is the reset): bits(f32((pcg(0x9E3779B9 ^ k) >> 8) / 2^24)),
    a Math.random()-like value; ranks g > 0 use pcg(seed_k ^ g*0x9E3779B9)."""
    s = int(np.array([(pcg((0x9E3779B9 ^ k) & 0xFFFFFFFF) >> 8) / 16777216.0],
                     dtype=np.float32).view(np.uint32)[0])
    if rank:
        s = pcg(s ^ ((rank * 0x9E3779B9) & 0xFFFFFFFF))
    return s


def seed_stream(n: int, start: int = 1, rank: int = 0) -> np.ndarray:
    return np.array([seed_bits(k, rank) for k in range(start, start + n)], dtype=np.uint32)


# ----------------------------------------------------------------- volumes
def sphere_in_cube(n: int = 64) -> np.ndarray:
    """py_notebooks/generate_test_volume.ipynb cell 1 at size n."""
    V = np.zeros((n, n, n), dtype=np.uint8)
    X, Y, Z = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n), np.linspace(-1, 1, n))
    V[X ** 2 + Y ** 2 + Z ** 2 < 0.5 ** 2] += 155
    V[np.maximum(np.abs(X), np.maximum(np.abs(Y), np.abs(Z))) < 0.8] += 100
    return V


def two_spheres(n: int = 64) -> np.ndarray:
    """generate_test_volume.ipynb cell 3 at size n. np.meshgrid's 'xy' axes
    (X along axis 1, Y along axis 0, Z along axis 2) by broadcasting: the same
    float64 values element for element, without three n^3 coordinate arrays."""
    V = np.zeros((n, n, n), dtype=np.uint8)
    t = np.linspace(-1, 1, n)
    X, Y, Z = t[None, :, None], t[:, None, None], t[None, None, :]
    V[X ** 2 + Y ** 2 + (Z - 0.5) ** 2 < 0.4 ** 2] += 200
    V[X ** 2 + Y ** 2 + (Z + 0.5) ** 2 < 0.4 ** 2] += 100
    return V


_synth = None


def _synth_lib():
    global _synth
    if _synth is None:
        p = LIB_DIR / "libvptsynth.so"
        if not p.exists():
            raise RuntimeError(f"{p} not built (run __graft_entry__.build())")
        _synth = C.CDLL(str(p))
        _synth.vs_fbm.restype = C.c_int
        _synth.vs_fbm.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.c_int, C.c_double, C.c_int]
        _synth.vs_noise3.restype = C.c_double
        _synth.vs_noise3.argtypes = [C.c_double, C.c_double, C.c_double, C.c_uint32]
    return _synth


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup") -> float | None:
    """CPUs' worth of time the process's cgroup may use (cpu.max quota / period,
    cgroup v2; cpu.cfs_quota_us / cpu.cfs_period_us, v1), or None if unlimited
    or unreadable. An affinity mask can list every CPU of the machine while the
    quota grants a few of them."""
    import math
    try:
        q, p = Path(root, "cpu.max").read_text().split()[:2]
        if q != "max" and int(p) > 0:
            return int(q) / int(p)
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(Path(root, "cpu", "cpu.cfs_quota_us").read_text())
        p = int(Path(root, "cpu", "cpu.cfs_period_us").read_text())
        return q / p if q > 0 and p > 0 and math.isfinite(q / p) else None
    except (OSError, ValueError):
        return None


def host_cpu_share() -> dict:
    """The host CPUs this process may use, by each limit that applies."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return {"affinity": aff, "cgroup_quota_cpus": cgroup_cpu_quota(),
            "omp_num_threads": int(omp) if omp.isdigit() and int(omp) > 0 else None,
            "os_cpu_count": os.cpu_count()}


def host_threads() -> int:
    """CPU threads the CPU baselines use: the CPUs this process may run on (its
    affinity mask), capped by the cgroup's CPU quota (rounded up) and by
    OMP_NUM_THREADS when the job sets them."""
    import math
    s = host_cpu_share()
    n = s["affinity"]
    if s["cgroup_quota_cpus"]:
        n = min(n, max(1, math.ceil(s["cgroup_quota_cpus"])))
    if s["omp_num_threads"]:
        n = min(n, s["omp_num_threads"])
    return max(1, n)


def fbm_volume(n: int, seed: int, octaves: int = 4, base_freq: float = 4.0,
               nthreads: int | None = None) -> np.ndarray:
    """PCG-lattice Perlin fBm (tools/vptsynth.c); C2: n=256 seed 1234, C3: n=512 seed 512,
    C5: n=1024 seed 1024."""
    out = np.empty((n, n, n), dtype=np.uint8)
    rc = _synth_lib().vs_fbm(C.c_void_p(out.ctypes.data), n, n, n, seed, octaves, base_freq,
                             nthreads or host_threads())
    if rc != 0:
        raise RuntimeError("vs_fbm failed")
    return out


# ----------------------------------------------------------------- tables
def tf_zero() -> np.ndarray:
    """The reference's default TF: a zero-filled texture (js:85, never uploaded)."""
    return np.zeros((256, 256, 4), dtype=np.uint8)


def tf_grey() -> np.ndarray:
    """C2: albedo 204, alpha = density ramp (row), b = 128 (g = +1/255), a = 0."""
    t = np.zeros((256, 256, 4), dtype=np.uint8)
    t[..., 0] = 204
    t[..., 1] = np.arange(256, dtype=np.uint8)[:, None]
    t[..., 2] = 128
    return t


def tf_spectral() -> np.ndarray:
    """C3: albedo(lambda) = .55 + .35 sin(2 pi 1.5 col/256), alpha = smoothstep(.15,.85,row/255),
    b = 217 (HG g = 0.702), a = 0."""
    col = np.arange(256, dtype=np.float64)
    row = np.arange(256, dtype=np.float64) / 255.0
    alb = np.round(255.0 * (0.55 + 0.35 * np.sin(2 * np.pi * 1.5 * col / 256.0)))
    x = np.clip((row - 0.15) / 0.7, 0.0, 1.0)
    alpha = np.round(255.0 * x * x * (3.0 - 2.0 * x))
    t = np.zeros((256, 256, 4), dtype=np.uint8)
    t[..., 0] = alb[None, :].astype(np.uint8)
    t[..., 1] = alpha[:, None].astype(np.uint8)
    t[..., 2] = 217
    return t


def tf_materials(varying_anisotropy: bool = True) -> np.ndarray:
    """A UI-like TF (MaterialTransferFunction.js:56-75 paints one material's
    256-entry albedo/alpha/anisotropy arrays into every density row of a range):
    three materials over density ranges; with varying_anisotropy the third
    material's anisotropy depends on wavelength (the general, non-row-invariant
    blue channel)."""
    t = np.zeros((256, 256, 4), dtype=np.uint8)
    col = np.arange(256)
    mats = [
        (slice(20, 90), 180, 60, np.full(256, 127)),
        (slice(90, 170), (150 + 80 * np.cos(col / 40.0)).astype(int), 140, np.full(256, 200)),
        (slice(170, 256), 230, 230,
         (60 + col * 0.7).astype(int) if varying_anisotropy else np.full(256, 30)),
    ]
    for rows, alb, alpha, aniso in mats:
        t[rows, :, 0] = alb
        t[rows, :, 1] = alpha
        t[rows, :, 2] = aniso
    return t


def light_default():
    """js:82-83: SPD 100 everywhere, direction [1, 0, 0]."""
    return np.full(256, 100, dtype=np.uint8), np.array([1.0, 0.0, 0.0], dtype=np.float32)


def algorithmic_bytes_per_pass(R: int, steps: int, nb: int = 12) -> int:
    """R^2 * (2*(40 + 4 nb) + 8 + 8 S)."""
    return R * R * (2 * (40 + 4 * nb) + 8 + 8 * steps)


def algorithmic_bytes_per_launch(R: int, steps: int, passes: int, nb: int = 12) -> int:
    """SURVEY 8(d), counting only what a launch materialises: a launch running
    `passes` passes back to back reads and writes the observable photon state
    once, gathers S 2x2x2 cells per photon per pass, and stores one rgba16f
    image (its last pass's: the passes of a launch are queued render() calls
    with no read between them): R^2 * (2*(40 + 4 nb) + 8 + passes*8 S).
    passes=1 is the per-pass formula."""
    return R * R * (2 * (40 + 4 * nb) + 8 + passes * 8 * steps)
