"""Pure-Python f32 restatement of the spectral MCM march — TEST INFRASTRUCTURE.

A second, independent restatement (numpy float32 scalars, Python-int u32
arithmetic), written directly from MCMSpectralComputeRenderer.wgsl and its
mixins, used only to cross-check the C oracle on small cases (a few pixels).
It follows the same arithmetic specification: f32 ops in WGSL
evaluation order with exactly the spec's listed products fused (fma32, an
exact rational fma rounded once to f32), the spec log/sin/cos polynomials,
explicit min/max, the software linear/clamp sampler.
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

F = np.float32
M32 = 0xFFFFFFFF
EPS = F(1e-5)
TWOPI = F(6.28318530718)
INV255 = F(1.0 / 255.0)


def bits(x) -> int:
    return int(np.array([x], np.float32).view(np.uint32)[0])


def fbits(u: int):
    return np.array([u & M32], np.uint32).view(np.float32)[0]


def pcg(v: int) -> int:  # pcg.wgsl:3-7
    v = int(v)
    x = (v * 747796405 + 2891336453) & M32
    x = (((x >> ((x >> 28) + 4)) ^ x) * 277803737) & M32
    return ((x >> 22) ^ x) & M32


def hash3(x: int, y: int, z: int) -> int:  # squashlinear.wgsl:7-9
    x, y, z = int(x), int(y), int(z)
    return pcg((19 * x + 47 * y + 101 * z + 131) & M32)


class Rng:
    def __init__(self, s: int):
        self.s = s & M32

    def uniform(self):  # uniformdivision.wgsl
        self.s = pcg(self.s)
        return F(self.s) / F(4294967296.0)


def fma32(a, b, c):
    """RN_f32(a*b + c) with a single rounding (exact rational arithmetic,
    then round-to-odd in double so the final f32 rounding is correct)."""
    a, b, c = F(a), F(b), F(c)
    if not (np.isfinite(a) and np.isfinite(b) and np.isfinite(c)):
        return F(float(a) * float(b) + float(c))
    x = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    if x == 0:
        # exact zero: the sign follows IEEE rules for the sum of the product and c
        p = float(a) * float(b)
        return F(p + float(c))
    d = float(x)
    if math.isfinite(d) and Fraction(d) != x and (np.array([d]).view(np.uint64)[0] & 1) == 0:
        d = float(np.nextafter(d, math.inf if Fraction(d) < x else -math.inf))
    return F(d)


def rcp(x):
    """Correctly rounded reciprocal RN(1/x): the spec's only true division."""
    return F(1) / F(x)


def smin(a, b):
    if a != a:
        return b
    if b != b:
        return a
    return b if b < a else a


def smax(a, b):
    if a != a:
        return b
    if b != b:
        return a
    return b if b > a else a


def spec_log(x):
    x = F(x)
    b = bits(x)
    if x != x or (b >> 31):
        return F(-np.inf) if x == 0 else F(np.nan)
    if x == 0:
        return F(-np.inf)
    if b == 0x7F800000:
        return x
    e = 0
    if b < 0x00800000:
        x = x * F(33554432.0)
        b = bits(x)
        e = -25
    e += (b >> 23) - 127
    m = fbits((b & 0x7FFFFF) | 0x3F800000)
    if m > F(1.41421353816986083984375):
        m = m * F(0.5)
        e += 1
    f = m - F(1)
    s = f / (F(2) + f)
    z = s * s
    P = fma32(z, fma32(z, fma32(z, fma32(z, F(0.1818181872367859), F(0.2222222238779068)),
                                 F(0.2857142984867096)), F(0.4000000059604645)), F(0.6666666865348816))
    R = z * P
    lm = fma32(s, R, s + s)
    ef = F(e)
    return fma32(ef, F(0.693115234375), fma32(ef, F(3.194618329871446e-05), lm))


def spec_sincos(x):
    x = F(x)
    kf = np.floor(fma32(x, F(0.6366197466850281), F(0.5)))
    r = fma32(-kf, F(7.549790126404332e-08),
              fma32(-kf, F(0.0004837512969970703), fma32(-kf, F(1.5703125), x)))
    z = r * r
    ps = fma32(z, fma32(z, fma32(z, fma32(z, F(-2.5052107943679403e-08), F(2.7557318844628753e-06)),
                                 F(-0.00019841270113829523)), F(0.008333333767950535)),
               F(-0.1666666716337204))
    s = fma32(r * z, ps, r)
    pc = fma32(z, fma32(z, fma32(z, F(-2.755731998149713e-07), F(2.4801587642286904e-05)),
                        F(-0.0013888889225199819)), F(0.0416666679084301))
    c = fma32(z * z, pc, fma32(F(-0.5), z, F(1)))
    k = int(kf) & 3
    return [(s, c), (c, -s), (-s, -c), (-c, s)][k]


def dot(a, b):
    return fma32(a[2], b[2], fma32(a[1], b[1], a[0] * b[0]))


def normalize(v):
    il = rcp(np.sqrt(dot(v, v)))
    return [v[0] * il, v[1] * il, v[2] * il]


def axis(u, n):
    u = F(u)
    u = u if u >= F(-1) else F(-1)
    u = u if u <= F(2) else F(2)
    x = fma32(u, F(n), F(-0.5))
    fl = np.floor(x)
    f = x - fl
    i = int(fl)
    return min(max(i, 0), n - 1), min(max(i + 1, 0), n - 1), f


def lerp(a, b, f):
    return fma32(f, b - a, a)


def tex3d(vol, p):
    D, H, W = vol.shape
    x0, x1, fx = axis(p[0], W)
    y0, y1, fy = axis(p[1], H)
    z0, z1, fz = axis(p[2], D)
    v = lambda i, j, k: F(int(vol[k, j, i]))  # noqa: E731
    c00 = lerp(v(x0, y0, z0), v(x1, y0, z0), fx)
    c10 = lerp(v(x0, y1, z0), v(x1, y1, z0), fx)
    c01 = lerp(v(x0, y0, z1), v(x1, y0, z1), fx)
    c11 = lerp(v(x0, y1, z1), v(x1, y1, z1), fx)
    return lerp(lerp(c00, c10, fy), lerp(c01, c11, fy), fz) * INV255


def tex2d_tf(tf, t, d):
    c0, c1, fx = axis(t, 256)
    r0, r1, fy = axis(d, 256)
    out = []
    for ch in range(3):
        a = lerp(F(int(tf[r0, c0, ch])), F(int(tf[r0, c1, ch])), fx)
        b = lerp(F(int(tf[r1, c0, ch])), F(int(tf[r1, c1, ch])), fx)
        out.append(lerp(a, b, fy) * INV255)
    return out


def tex_light(light, t):
    c0, c1, fx = axis(t, 256)
    return lerp(F(int(light[c0])), F(int(light[c1])), fx) * INV255


class Photon:
    def __init__(self, words):
        w = np.asarray(words, np.uint32)
        f = w.view(np.float32)
        self.position = [f[0], f[1], f[2]]
        self.bounces = int(w[3])
        self.direction = [f[4], f[5], f[6]]
        self.samples = int(w[7])
        self.bin = int(w[8])
        self.wavelength = f[9]
        self.radiance = [f[10 + i] for i in range(12)]

    def words(self):
        w = np.zeros(36, np.uint32)
        f = w.view(np.float32)
        f[0:3] = self.position
        w[3] = self.bounces & M32
        f[4:7] = self.direction
        w[7] = self.samples & M32
        w[8] = self.bin & M32
        f[9] = self.wavelength
        f[10:22] = self.radiance
        f[22:34] = F(1)
        return w


class Ref:
    """One renderer's inputs; render_pixel / reset_pixel follow compute_main."""

    def __init__(self, R, spectrum, mvp, volume=None, tf=None, light=None, light_dir=(1, 0, 0),
                 extinction=1.0, bounces=8, steps=8, blur=0.0):
        self.R = R
        self.spec = np.asarray(spectrum, np.float32)
        self.m = np.asarray(mvp, np.float32).reshape(16)
        self.vol, self.tf, self.light = volume, tf, light
        self.light_dir = [F(v) for v in light_dir]
        self.ext, self.maxb, self.steps, self.blur = F(extinction), bounces, steps, F(blur)
        self.inv = F(1.0 / R)

    def nb(self):
        v = self.spec[0] + F(0.5)
        return int(v) if v > 0 else 0

    def screen(self, x, y):  # wgsl:118
        return (fma32(F(x) + F(0.5), self.inv, F(-0.5)) * F(2),
                fma32(F(y) + F(0.5), self.inv, F(-0.5)) * F(-2))

    def mat_vec(self, v):
        m = self.m
        return [fma32(m[12 + r], v[3], fma32(m[8 + r], v[2], fma32(m[4 + r], v[1], m[r] * v[0])))
                for r in range(4)]

    def disk(self, rng):
        radius = np.sqrt(rng.uniform())
        angle = TWOPI * rng.uniform()
        s, c = spec_sincos(angle)
        return radius * c, radius * s

    def reset(self, p, screen, rng):  # PhotonSpectral_reset, wgsl:249-266
        dx, dy = self.disk(rng)
        nearp = [fma32(dx, self.blur, screen[0]), fma32(dy, self.blur, screen[1]), F(-1), F(1)]
        sqx, sqy = rng.uniform(), rng.uniform()
        farp = [fma32(fma32(sqx, F(2), F(-1)), self.inv, screen[0]),
                fma32(fma32(sqy, F(2), F(-1)), self.inv, screen[1]), F(1), F(1)]
        fd, td = self.mat_vec(nearp), self.mat_vec(farp)
        iw, jw = rcp(fd[3]), rcp(td[3])
        frm = [fd[0] * iw, fd[1] * iw, fd[2] * iw]
        to = [td[0] * jw, td[1] * jw, td[2] * jw]
        d = normalize([to[0] - frm[0], to[1] - frm[1], to[2] - frm[2]])
        p.direction = d
        p.bounces = 0
        rd = [rcp(d[i]) for i in range(3)]
        t1 = [smin((F(0) - frm[i]) * rd[i], (F(1) - frm[i]) * rd[i]) for i in range(3)]
        tn = smax(smax(smax(t1[0], t1[1]), t1[2]), F(0))
        p.position = [fma32(tn, d[i], frm[i]) for i in range(3)]
        nb = self.nb()
        lo, hi = self.spec[1], self.spec[nb + 1]
        lam = fma32(rng.uniform(), hi - lo, lo)
        p.wavelength = lam
        p.bin = (nb - 1) & M32
        for i in range(1, nb):
            if lam < self.spec[i + 1]:
                p.bin = i - 1
                break

    def reset_pixel(self, x, y, seed):
        p = Photon(np.zeros(36, np.uint32))
        rng = Rng(hash3(x, y, seed))
        self.reset(p, self.screen(x, y), rng)
        p.samples = 0
        p.radiance = [F(1)] * 12
        return p

    def add_radiance(self, p, L):
        inv_n = rcp(F(p.samples))
        for i in range(min(self.nb(), 12)):
            tgt = L if i == p.bin else F(0)
            p.radiance[i] = fma32(tgt - p.radiance[i], inv_n, p.radiance[i])

    def render_pixel(self, p, x, y, seed):
        screen = self.screen(x, y)
        rng = Rng(hash3(x, y, seed))
        for _ in range(self.steps):
            dist = -spec_log(rng.uniform()) * rcp(self.ext)
            p.position = [fma32(dist, p.direction[i], p.position[i]) for i in range(3)]
            dens = tex3d(self.vol, p.position)
            t = (p.wavelength - F(400)) * rcp(F(700) - F(400))
            albedo, alpha, b = tex2d_tf(self.tf, t, dens)
            aniso = b * F(2) - F(1)
            pnull = F(1) - alpha
            pscat = F(0) if p.bounces >= self.maxb else alpha * albedo
            pabs = (F(1) - pnull) - pscat
            wheel = rng.uniform()
            pos = p.position
            if pos[0] > 1 or pos[1] > 1 or pos[2] > 1 or pos[0] < 0 or pos[1] < 0 or pos[2] < 0:
                intensity = tex_light(self.light, t) * F(5)
                ld = self.light_dir
                if np.sqrt(dot(ld, ld)) < EPS:
                    rad = intensity
                else:
                    rad = smax(dot(p.direction, normalize(ld)) * intensity, F(0))
                p.samples += 1
                self.add_radiance(p, rad)
                self.reset(p, screen, rng)
            elif wheel < pabs:
                p.samples += 1
                self.add_radiance(p, F(0))
                self.reset(p, screen, rng)
            elif wheel < pabs + pscat:
                p.direction = self.hg(rng, aniso, p.direction)
                p.bounces += 1
        nb = self.nb()
        X = Y = Z = F(0)
        for i in range(min(nb, 12)):
            X = fma32(p.radiance[i], self.spec[2 + nb + i], X)
            Y = fma32(p.radiance[i], self.spec[2 + 2 * nb + i], Y)
            Z = fma32(p.radiance[i], self.spec[2 + 3 * nb + i], Z)
        rgb = [fma32(F(-0.498536), Z, fma32(F(-1.537150), Y, F(3.240479) * X)),
               fma32(F(0.041556), Z, fma32(F(1.875990), Y, F(-0.969255) * X)),
               fma32(F(1.057311), Z, fma32(F(-0.204041), Y, F(0.055647) * X))]
        return rgb

    def hg(self, rng, g, d):  # wgsl:82-97
        dx, dy = self.disk(rng)
        nrm = fma32(dy, dy, dx * dx)
        radius = F(2) * np.sqrt(F(1) - nrm)
        u = [radius * dx, radius * dy, F(1) - F(2) * nrm]
        if abs(g) < EPS:
            return u
        g2 = g * g
        c = (F(1) - g2) * rcp(fma32(F(2) * g, rng.uniform(), F(1) - g))
        cos = fma32(-c, c, F(1) + g2) * rcp(F(2) * g)
        ud = dot(u, d)
        circle = normalize([fma32(-ud, d[i], u[i]) for i in range(3)])
        sn = np.sqrt(fma32(-cos, cos, F(1)))
        return [fma32(sn, circle[i], cos * d[i]) for i in range(3)]
