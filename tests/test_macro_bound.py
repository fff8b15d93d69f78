"""The macro-cell alpha bound's arithmetic, proved on the CPU.

A march step skips its volume gather when its wheel value is at least the
threshold of its macro cell (csrc/kernels.hip maj_threshold, k_macro_minmax,
k_macro_alpha; host table sizing in csrc/vptmcm.cpp volume_begin_one). That is
only legal when every outcome the skipped sample could have produced is the
null collision, i.e. threshold >= pabs + pscat as the reference computes them
(MCMSpectralComputeRenderer.wgsl:132-139: pnull = 1 - alpha, pscat = alpha *
albedo, pabs = 1 - pnull - pscat; wheel < pabs absorbs, < pabs + pscat
scatters). Three links, each checked here in f32 as the kernel rounds:
  1. the TF rows a sample can touch lie in [vmin - 2, vmax + 2] of its macro
     cell's voxel bytes (trilinear filter, then the TF's row axis);
  2. the macro cell the kernel looks up covers both corner voxels of the
     texel cell it gathers, for every cell of ragged and power-of-two sizes;
  3. with alpha from a bilinear lerp of bytes <= k and q = ceil(k / 17),
     fma(17 q, RN(1/255), 2^-16) exceeds pabs and pabs + pscat for every
     albedo.
The RGB sibling (k_march_rgb, MCMComputeRenderer.wgsl) gets the same bound
from row 0 of its TF: the last two tests. The GPU side (tests/test_gpu_fuzz.py
even cases, test_gpu_knobs.py and test_gpu_rgb.py with VPTMCM_MAJ=on) checks
the whole march bit-exact against the oracle with it.
"""
import numpy as np

F32 = np.float32
INV255 = F32(1.0) / F32(255.0)
KMAJ_BYTES = 20480  # csrc/march.h kMajBytes


def rn(x):
    return np.asarray(x, np.float64).astype(F32)


def fma(a, b, c):
    """RN_f32(a*b + c): the f64 product of two f32 is exact; the f64 sum can
    round once before the f32 rounding (a 1-ulp risk far inside every margin
    below)."""
    return rn(np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64))


def lerp(a, b, f):  # csrc/mcm_device.h lerp: fma(f, b - a, a)
    return fma(f, (F32(b) if np.isscalar(b) else b) - a, a)


def threshold(q):  # kernels.hip maj_threshold
    return fma(F32(q * 17), INV255, F32(2.0 ** -16))


def test_rows_a_sample_reaches_stay_within_two_of_its_bytes():
    rng = np.random.default_rng(1)
    n = 400_000
    vmin = rng.integers(0, 256, n)
    vmax = np.minimum(vmin + rng.integers(0, 256, n), 255)
    span = (vmax - vmin + 1).astype(np.float64)
    b = (vmin[:, None] + np.floor(rng.random((n, 8)) * span[:, None])).astype(np.int64)
    b[: n // 8] = vmin[: n // 8, None]  # flat cells at either end of the range
    b[n // 8: n // 4] = vmax[n // 8: n // 4, None]
    fr = rng.random((n, 3)).astype(F32)
    fr[: n // 16] = F32(1.0)
    fr[n // 16: n // 8] = F32(0.0)
    c = b.astype(F32)
    c00 = lerp(c[:, 0], c[:, 1], fr[:, 0])
    c10 = lerp(c[:, 2], c[:, 3], fr[:, 0])
    c01 = lerp(c[:, 4], c[:, 5], fr[:, 0])
    c11 = lerp(c[:, 6], c[:, 7], fr[:, 0])
    d = lerp(lerp(c00, c10, fr[:, 1]), lerp(c01, c11, fr[:, 1]), fr[:, 2]) * INV255  # vol_filter
    x = fma(np.clip(d, F32(-1), F32(2)), F32(256.0), F32(-0.5))  # the TF's row axis
    i = np.floor(x).astype(np.int64)
    r0, r1 = np.clip(i, 0, 255), np.clip(i + 1, 0, 255)
    lo, hi = np.maximum(vmin - 2, 0), np.minimum(vmax + 2, 255)  # k_macro_alpha's rows
    assert np.all(r0 >= lo) and np.all(r1 <= hi)


def test_macro_cell_covers_the_gathered_cell():
    for W in (1, 2, 7, 8, 9, 31, 39, 44, 64, 255, 256, 257, 512, 1023, 1024):
        for s in range(3, 11):
            nx = (W + (1 << s)) >> s  # ceil((W + 1) / 2^s), vptmcm.cpp
            for c in range(0, W + 1):  # clampi(ix + 1, W): every texel cell
                m = c >> s
                assert m < nx
                lo = max((m << s) - 1, 0)  # k_macro_minmax's voxel range
                hi = min(((m + 1) << s) - 1, W - 1)
                for v in (min(max(c - 1, 0), W - 1), min(c, W - 1)):  # the cell's corner voxels
                    assert lo <= v <= hi, (W, s, c, m)


def test_table_sizes():
    """The finest power-of-two macro (>= 8 cells) whose 4-bit codes fit the
    LDS table: 512^3 -> 16-cell macros (33^3 codes), 1024^3 -> 32."""
    def pick(W, H, D):
        for s in range(3, 14):
            n = ((W + (1 << s)) >> s) * ((H + (1 << s)) >> s) * ((D + (1 << s)) >> s)
            if ((n + 1) // 2 + 15) // 16 * 16 <= KMAJ_BYTES:
                return s, n
        return None
    assert pick(512, 512, 512) == (4, 33 ** 3)
    assert pick(1024, 1024, 1024) == (5, 33 ** 3)
    assert pick(64, 64, 64) == (3, 9 ** 3)
    assert pick(31, 44, 39)[0] == 3


def test_threshold_dominates_pabs_and_pscat():
    rng = np.random.default_rng(2)
    albedo = np.concatenate([
        np.arange(256, dtype=F32) * INV255, rng.random(512).astype(F32),
        np.array([0.0, 1.0, np.nextafter(F32(1), F32(2))], F32)])
    worst = np.inf
    for k in range(256):
        q = (k + 16) // 17  # k_macro_alpha
        thr = threshold(q)
        kf = F32(k)
        # the outer TF lerp of two inner lerps of bytes <= k, sampled
        ap = (rng.random(4096) * k).astype(F32)
        bp = (rng.random(4096) * k).astype(F32)
        ap[:64], bp[64:128] = kf, kf
        fy = rng.random(4096).astype(F32)
        fy[::7] = F32(1.0)
        top = lerp(ap, bp, fy)
        cap = np.nextafter(kf, F32(np.inf))
        assert np.all(top <= cap)
        # every f32 alpha value up to the cap's (the top 256 exhaustively)
        hi = rn(cap * INV255)
        near = (hi.view(np.uint32) - np.arange(256, dtype=np.uint32)).view(F32)
        alpha = np.concatenate([near[near >= 0], (top * INV255).astype(F32)])
        a = alpha[:, None]
        pnull = F32(1) - a
        for pscat in (np.zeros_like(a), a * albedo[None, :]):  # bounces exhausted or not
            pabs = (F32(1) - pnull) - pscat
            tot = pabs + pscat
            assert np.all(tot < thr) and np.all(pabs < thr), (k, q)
            worst = min(worst, float(np.min(thr.astype(np.float64) - tot.astype(np.float64))))
    assert worst > 2.0 ** -18  # the margin the 2^-16 term buys


def rgb_rowmax(alpha_bytes: np.ndarray) -> np.ndarray:
    """vptmcm.cpp set_transfer_function_one: per density byte v the largest
    alpha byte of TF row 0's texels [floor((v-1)/255 w - 0.5) - 1,
    floor((v+1)/255 w - 0.5) + 2], clamped."""
    w = len(alpha_bytes)
    out = np.zeros(256, np.uint8)
    for v in range(256):
        lo = max(0, int(np.floor((v - 1) / 255.0 * w - 0.5)) - 1)
        hi = min(w - 1, int(np.floor((v + 1) / 255.0 * w - 0.5)) + 2)
        out[v] = alpha_bytes[lo:hi + 1].max()
    return out


def test_rgb_texels_a_sample_reaches_are_in_its_rows():
    """The RGB sibling samples TF row 0 at (density, 0) (MCMComputeRenderer.wgsl
    sampleVolumeColor; kernels.hip k_march_rgb): texels floor(d w - 0.5) and
    the next, clamped. Every alpha byte it can read is within the macro cell's
    code (the row maxima of bytes vmin - 2 .. vmax + 2, k_macro_alpha)."""
    rng = np.random.default_rng(3)
    for w in (2, 3, 100, 255, 256, 257, 1000, 4096):
        alpha = rng.integers(0, 256, w).astype(np.uint8)
        rm = rgb_rowmax(alpha)
        n = 100_000
        vmin = rng.integers(0, 256, n)
        vmax = np.minimum(vmin + rng.integers(0, 64, n), 255)
        span = (vmax - vmin + 1).astype(np.float64)
        b = (vmin[:, None] + np.floor(rng.random((n, 8)) * span[:, None])).astype(F32)
        fr = rng.random((n, 3)).astype(F32)
        c00, c10 = lerp(b[:, 0], b[:, 1], fr[:, 0]), lerp(b[:, 2], b[:, 3], fr[:, 0])
        c01, c11 = lerp(b[:, 4], b[:, 5], fr[:, 0]), lerp(b[:, 6], b[:, 7], fr[:, 0])
        d = lerp(lerp(c00, c10, fr[:, 1]), lerp(c01, c11, fr[:, 1]), fr[:, 2]) * INV255
        x = fma(np.clip(d, F32(-1), F32(2)), F32(w), F32(-0.5))
        i = np.floor(x).astype(np.int64)
        got = np.maximum(alpha[np.clip(i, 0, w - 1)], alpha[np.clip(i + 1, 0, w - 1)])
        code_k = np.array([rm[max(a - 2, 0):min(c + 2, 255) + 1].max() for a, c in zip(vmin, vmax)])
        assert np.all(got <= code_k), w


def test_rgb_threshold_dominates_pabs_and_pscat():
    """alpha = lerp of two RN(byte / 255) texels (the host decodes alpha
    linearly), pscat = alpha * max(r, g, b) with the sRGB-decoded channels
    (<= 1, one ulp over allowed)."""
    rng = np.random.default_rng(4)
    cmax = np.concatenate([rng.random(512).astype(F32),
                           np.array([0.0, 1.0, np.nextafter(F32(1), F32(2))], F32)])
    for k in range(256):
        thr = threshold((k + 16) // 17)
        a = (rng.integers(0, k + 1, 4096).astype(F32) * INV255).astype(F32)
        bb = (rng.integers(0, k + 1, 4096).astype(F32) * INV255).astype(F32)
        a[:64] = bb[64:128] = F32(k) * INV255
        ft = rng.random(4096).astype(F32)
        ft[::5] = F32(1.0)
        ca = lerp(a, bb, ft)[:, None]
        pnull = F32(1) - ca
        for pscat in (np.zeros_like(ca), ca * cmax[None, :]):
            pabs = (F32(1) - pnull) - pscat
            assert np.all(pabs + pscat < thr) and np.all(pabs < thr), k
