"""CPU tests of the oracle: known answers, spec-math accuracy, golden fixtures,
and cross-checks against the independent pure-Python restatement (pyref)."""
import json
import math
from pathlib import Path

import numpy as np
import pytest

import oracle as orc
import pyref
from vptmcm import configs as cf

GOLD = Path(__file__).resolve().parent / "golden"


def test_pcg_known_answers(oracle_lib):
    # SURVEY §8 a9 — computed from pcg.wgsl:3-7 / squashlinear.wgsl:7-9
    assert oracle_lib.orc_hash(0) == 129708002
    assert oracle_lib.orc_hash(1) == 2831084092
    s = oracle_lib.orc_hash3(0, 0, 0x3F000000)
    assert s == 3111607799
    us = []
    for _ in range(4):
        s = oracle_lib.orc_hash(s)
        us.append(np.float32(s) / np.float32(4294967296.0))
    np.testing.assert_allclose(us, [0.83673555, 0.50443858, 0.22452752, 0.81816036], atol=5e-8)
    assert pyref.pcg(0) == 129708002 and pyref.hash3(0, 0, 0x3F000000) == 3111607799


def _ulp(x: np.ndarray) -> np.ndarray:
    x = np.abs(x.astype(np.float32))
    return (np.nextafter(x, np.float32(np.inf)) - x).astype(np.float64)


def test_spec_log_accuracy():
    o = orc.Oracle(1)
    rng = np.random.default_rng(0)
    # the kernel's inputs: u = f32(state) * 2^-32 for u32 states, plus edges
    states = rng.integers(1, 2 ** 32, 400_000, dtype=np.uint64)
    u = (states.astype(np.float32) * np.float32(2.0 ** -32)).astype(np.float32)
    u = np.concatenate([u, np.float32([1.0, 0.5, 2.0 ** -32, 1e-38, 1e-45, 3.0, 1e30])])
    got = o.eval_batch(0, u.view(np.uint32)).view(np.float32).astype(np.float64)
    ref = np.log(u.astype(np.float64))
    err = np.abs(got - ref) / _ulp(ref)
    assert err.max() <= 2.0, f"log max ulp {err.max()}"   # WGSL allows 3 ULP
    edge = o.eval_batch(0, np.float32([0.0, -0.0, -1.0, np.inf, np.nan]).view(np.uint32))
    e = edge.view(np.float32)
    assert e[0] == -np.inf and e[1] == -np.inf and np.isnan(e[2]) and e[3] == np.inf and np.isnan(e[4])


def test_spec_sincos_accuracy():
    o = orc.Oracle(1)
    x = np.linspace(0.0, 6.2831855, 300_001, dtype=np.float32)
    s = o.eval_batch(1, x.view(np.uint32)).view(np.float32).astype(np.float64)
    c = o.eval_batch(2, x.view(np.uint32)).view(np.float32).astype(np.float64)
    xd = x.astype(np.float64)
    assert np.abs(s - np.sin(xd)).max() < 2e-7      # WGSL allows 2^-11 absolute
    assert np.abs(c - np.cos(xd)).max() < 2e-7
    big = np.abs(np.sin(xd)) > 1e-3
    assert (np.abs(s - np.sin(xd))[big] / _ulp(np.sin(xd))[big]).max() <= 2.0


def test_f16_rounding_matches_ieee():
    o = orc.Oracle(1)
    rng = np.random.default_rng(1)
    x = np.concatenate([
        rng.standard_normal(200_000).astype(np.float32) * np.float32(100.0),
        (rng.random(50_000) * 1e-4).astype(np.float32),            # f16 subnormal range
        np.float32([65504.0, 65519.99, 65520.0, 1e9, -1e9, 0.0, -0.0, 6e-8, 2.98e-8, np.inf, -np.inf]),
    ])
    got = o.eval_batch(4, x.view(np.uint32)).astype(np.uint16)
    want = x.astype(np.float16).view(np.uint16)
    assert np.array_equal(got, want)
    nan = o.eval_batch(4, np.float32([np.nan]).view(np.uint32))
    assert np.isnan(np.uint16(nan[0]).view(np.float16))


def test_sampler_known_answers(oracle_lib):
    import ctypes as C
    vol = np.zeros((4, 4, 4), np.uint8)
    vol[1, 2, 3] = 255          # z=1, y=2, x=3
    def sv(p):
        pp = (C.c_float * 3)(*p)
        return oracle_lib.orc_sample_volume(C.c_void_p(vol.ctypes.data), 4, 4, 4, pp)
    # texel centre (x=3 -> (3+.5)/4) returns exactly 1
    assert sv([3.5 / 4, 2.5 / 4, 1.5 / 4]) == 1.0
    # half way between two texel centres along x: 0.5 of the value
    assert abs(sv([3.0 / 4, 2.5 / 4, 1.5 / 4]) - 0.5) < 1e-7
    # clamp-to-edge: beyond the last centre stays at the edge texel
    assert sv([1.5, 2.5 / 4, 1.5 / 4]) == 1.0
    # NaN coordinate is sanitised to the low edge (texel 0 on that axis)
    assert sv([3.5 / 4, 2.5 / 4, float("nan")]) == 0.0
    tf = np.zeros((256, 256, 4), np.uint8)
    tf[10, 20] = (255, 128, 64, 0)       # row 10 (density), column 20 (wavelength)
    out = (C.c_float * 3)()
    oracle_lib.orc_sample_tf(C.c_void_p(tf.ctypes.data), (20 + 0.5) / 256, (10 + 0.5) / 256, out)
    assert list(out) == [1.0, np.float32(128) * np.float32(1 / 255), np.float32(64) * np.float32(1 / 255)]


def test_golden_spectrum_buffer_matches_survey():
    buf = cf.spectrum_buffer("12")
    assert buf[0] == 12 and list(buf[1:14]) == list(range(400, 701, 25))
    x = [0.0734938, 0.3159133, 0.2634736, 0.0567988, 0.0292408, 0.2557066, 0.6287991, 0.9829873,
         0.9574324, 0.5108532, 0.1567253, 0.0319270]
    y = [0.0021791, 0.0200807, 0.0679036, 0.1935324, 0.5478964, 0.9180674, 0.9785573, 0.7883375,
         0.4797107, 0.2056333, 0.0581967, 0.0115880]
    z = [0.3524810, 1.5806301, 1.5453538, 0.5935612, 0.1484911, 0.0284939, 0.0040373, 0.0013103,
         0.0003760, 0.0000329, 0, 0]
    np.testing.assert_allclose(buf[14:26], x, atol=1e-6)
    np.testing.assert_allclose(buf[26:38], y, atol=1e-6)
    np.testing.assert_allclose(buf[38:50], z, atol=1e-6)
    assert not buf[50:].any()


def test_golden_mvp_matches_configs():
    d = json.loads((GOLD / "mvp_inverse.json").read_text())
    assert d["cameras"]["default"]["bits"] == [int(b) for b in cf.DEFAULT_MVP_INVERSE_BITS]


def _setup_pair(R, vol, tf, spec, ext, light_dir=(1, 0, 0), bounces=8, steps=8, blur=0.0,
                mvp=None):
    mvp = cf.default_mvp_inverse() if mvp is None else mvp
    spd = np.full(256, 100, np.uint8)
    o = orc.Oracle(R)
    o.set_spectrum(spec)
    o.volume, o.tf, o.light = vol, tf, spd
    o.light_dir = np.asarray(light_dir, np.float32)
    o.params.update(extinction=ext, bounces=bounces, steps=steps, blur=blur)
    p = pyref.Ref(R, o.spectrum, mvp, vol, tf, spd, light_dir, ext, bounces, steps, blur)
    return o, p, mvp


def _cmp_words(a: np.ndarray, b: np.ndarray) -> bool:
    fa, fb = a.view(np.float32), b.view(np.float32)
    return bool(((a == b) | (np.isnan(fa) & np.isnan(fb))).all())


@pytest.mark.parametrize("case", ["sphere_tf3_ext1", "sphere_tf3_ext32", "fbm_grey_ext32",
                                  "two_spheres_iso_light", "zero_tf", "bounces0_blur"])
def test_oracle_matches_pyref(case):
    """The C oracle and the independent Python restatement agree bit for bit."""
    R = 8
    spec = cf.spectrum_buffer("12")
    if case.startswith("sphere"):
        vol, tf, ext = cf.sphere_in_cube(16), cf.tf_spectral(), 1.0 if case.endswith("1") else 32.0
        kw = {}
    elif case == "fbm_grey_ext32":
        vol, tf, ext, kw = cf.fbm_volume(16, 1234, nthreads=2), cf.tf_grey(), 32.0, {}
    elif case == "two_spheres_iso_light":
        vol, tf, ext, kw = cf.two_spheres(16), cf.tf_spectral(), 8.0, {"light_dir": (0, 0, 0)}
    elif case == "zero_tf":
        vol, tf, ext, kw = cf.sphere_in_cube(16), cf.tf_zero(), 1.0, {}
    else:
        vol, tf, ext = cf.sphere_in_cube(16), cf.tf_spectral(), 16.0
        kw = {"bounces": 0, "blur": 0.05, "mvp": cf.golden_mvp("orbit_tilted")}
    o, p, mvp = _setup_pair(R, vol, tf, spec, ext, **kw)
    seeds = cf.seed_stream(3, start=0)
    o.reset(mvp, seeds[0])
    ph = [p.reset_pixel(x, y, seeds[0]) for y in range(R) for x in range(R)]
    assert _cmp_words(o.photons, np.stack([q.words() for q in ph]))
    for s in seeds[1:]:
        rgb_o, _ = o.render(mvp, s)
        for y in range(R):
            for x in range(R):
                rgb = p.render_pixel(ph[y * R + x], x, y, s)
                assert np.array_equal(np.float32(rgb), rgb_o[y, x]) or \
                    np.isnan(rgb).any(), (case, x, y)
        assert _cmp_words(o.photons, np.stack([q.words() for q in ph])), case


def test_first_reset_quirk():
    """Reset before any spectrum upload: n_bins = 0, wavelength 0,
    bin = 0xFFFFFFFF; the first render credits no bin."""
    R = 8
    o = orc.Oracle(R)
    mvp = cf.default_mvp_inverse()
    o.reset(mvp, cf.seed_bits(0))
    w = o.photons
    assert (w[:, 8] == 0xFFFFFFFF).all()
    assert (w[:, 9].view(np.float32) == 0).all()
    o.set_spectrum(cf.spectrum_buffer("12"))
    o.volume, o.tf, o.light = cf.sphere_in_cube(16), cf.tf_zero(), np.full(256, 100, np.uint8)
    o.params.update(extinction=1.0, steps=64)
    o.render(mvp, cf.seed_bits(1))
    first = o.photons
    assert (first[:, 7] >= 1).all()        # every photon exits at least once in 64 steps


def test_oracle_regression_fixture():
    """Pins the oracle's own output (any change to the spec must be deliberate)."""
    import hashlib
    R = 32
    o, _, mvp = _setup_pair(R, cf.sphere_in_cube(64), cf.tf_spectral(), cf.spectrum_buffer("12"), 32.0)
    seeds = cf.seed_stream(3, start=0)
    o.reset(mvp, seeds[0])
    for s in seeds[1:]:
        _, rgba = o.render(mvp, s)
    h = hashlib.sha256(o.photons.tobytes() + rgba.tobytes()).hexdigest()
    ref = json.loads((GOLD / "oracle_regression.json").read_text())
    assert h == ref["sha256_R32_sphere64_tf3_ext32_2pass"]


def test_tonemap_oracle_known_answers():
    """Identity settings (low 0, high 1, mid 0.5, gamma 1: exponent 1,
    saturation 1) quantise the clamped input; saturation 0 gives grey;
    negative / NaN inputs map to 0 (pow of a negative base is NaN in WGSL)."""
    o = orc.Oracle(1)
    v = np.float16([[0.0, 0.25, 1.0, 1.0], [2.0, -0.5, 0.5, 1.0], [np.nan, 0.1, 0.9, 1.0]])
    out = o.tonemap_artistic(v.view(np.uint16), gamma=1.0)
    assert out[0].tolist() == [0, 64, 255, 255]
    assert out[1, 0] == 255 and out[1, 1] == 0 and out[1, 2] == 128
    assert out[2, 0] == 0
    grey = o.tonemap_artistic(v.view(np.uint16)[:1], saturation=0.0, gamma=1.0)
    assert grey[0, 0] == grey[0, 1] == grey[0, 2] == round(255 * (0.0 + 0.25 + 1.0) / 3)


def test_rgb_oracle_srgb_decode_and_reset():
    """sRGB decode endpoints/midpoints (IEC 61966-2-1) and the RGB reset kernel's
    state: transmittance 1, radiance 1, samples 0, rays starting on the cube."""
    o = orc.OracleRGB(8)
    f = o.L.orc_srgb_to_linear
    assert f(0) == 0.0 and f(255) == 1.0
    assert abs(f(10) - (10 / 255) / 12.92) < 1e-9
    assert abs(f(128) - ((128 / 255 + 0.055) / 1.055) ** 2.4) < 1e-7
    o.reset(cf.default_mvp_inverse(), cf.seed_bits(0))
    w = o.photons
    fl = w.view(np.float32)
    assert (fl[:, 8:11] == 1.0).all() and (fl[:, 12:15] == 1.0).all()
    assert (w[:, 7] == 0).all() and (w[:, 3] == 0).all()
    assert np.allclose(np.linalg.norm(fl[:, 4:7], axis=1), 1.0, atol=1e-6)
