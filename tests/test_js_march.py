"""The JavaScript re-execution of the march (oracle/mcm_march.js, bench.py's
primary CPU baseline) against the C oracle: photons (all 36 words), the fp32
radiance_to_rgb image and the rgba16float image, bit for bit, over the
scenario families of test_oracle_matches_pyref plus the benchmark's own
inputs (fBm volume, spectral TF, default camera) and the first-reset quirk."""
import numpy as np
import pytest

import js_march
import oracle as orc
from vptmcm import configs as cf

pytestmark = pytest.mark.skipif(js_march.node() is None, reason="node not on PATH")


def _same(a, b):
    fa, fb = a.view(np.float32), b.view(np.float32)
    return (a == b) | (np.isnan(fa) & np.isnan(fb))


CASES = {
    "sphere_tf_spectral_ext1": dict(vol=lambda: cf.sphere_in_cube(16), tf=cf.tf_spectral, ext=1.0),
    "sphere_tf_spectral_ext32": dict(vol=lambda: cf.sphere_in_cube(16), tf=cf.tf_spectral, ext=32.0),
    "fbm_grey_ext32": dict(vol=lambda: cf.fbm_volume(16, 1234, nthreads=2), tf=cf.tf_grey, ext=32.0),
    "two_spheres_iso_light": dict(vol=lambda: cf.two_spheres(16), tf=cf.tf_spectral, ext=8.0,
                                  light_dir=(0.0, 0.0, 0.0)),
    "zero_tf": dict(vol=lambda: cf.sphere_in_cube(16), tf=cf.tf_zero, ext=1.0),
    "bounces0_blur_orbit": dict(vol=lambda: cf.sphere_in_cube(16), tf=cf.tf_spectral, ext=16.0,
                                bounces=0, blur=0.05, mvp="orbit_tilted"),
    "materials_uneven_bins": dict(vol=lambda: cf.fbm_volume(24, 7, nthreads=2),
                                  tf=lambda: cf.tf_materials(True), ext=24.0, spec="8_uneven",
                                  mvp="orbit"),
    "bench_inputs": dict(vol=lambda: cf.fbm_volume(32, 512, nthreads=2), tf=cf.tf_spectral,
                         ext=32.0, R=32),
}


@pytest.mark.parametrize("case", list(CASES))
def test_js_march_matches_c_oracle(case):
    c = CASES[case]
    R = c.get("R", 16)
    vol, tf = c["vol"](), c["tf"]()
    spd, ld = cf.light_default()
    ld = np.asarray(c.get("light_dir", ld), np.float32)
    spec = cf.spectrum_buffer(c.get("spec", "12"))
    mvp = cf.golden_mvp(c["mvp"]) if "mvp" in c else cf.default_mvp_inverse()
    kw = dict(extinction=c["ext"], bounces=c.get("bounces", 8), steps=8, blur=c.get("blur", 0.0))
    seeds = cf.seed_stream(4, start=3)

    o = orc.Oracle(R)
    o.set_spectrum(spec)
    o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
    o.params.update(**kw)
    o.reset(mvp, seeds[0])
    for s in seeds[1:]:
        rgb, rgba = o.render(mvp, s)

    ph, jrgb, jrgba = js_march.run_check(R, vol, tf, spd, ld, spec, mvp, seeds, threads=3, **kw)
    bad = ~_same(ph, o.photons)
    assert not bad.any(), f"{case}: {int(bad.sum())} photon words differ, first {np.argwhere(bad)[:4]}"
    assert _same(jrgb.view(np.uint32), rgb.view(np.uint32)).all(), f"{case}: fp32 rgb differs"
    assert np.array_equal(jrgba, rgba), f"{case}: rgba16f differs"


def test_js_march_first_reset_quirk():
    """Reset before any spectrum upload: n_bins 0, wavelength 0, bin 0xFFFFFFFF."""
    R = 8
    spd, ld = cf.light_default()
    vol, tf, mvp = cf.sphere_in_cube(16), cf.tf_spectral(), cf.default_mvp_inverse()
    seeds = cf.seed_stream(2, start=0)
    zero = np.zeros(64, np.float32)
    ph, _, _ = js_march.run_check(R, vol, tf, spd, ld, zero, mvp, seeds, threads=2,
                                  extinction=4.0)
    o = orc.Oracle(R)
    o.set_spectrum(zero)
    o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
    o.params.update(extinction=4.0, bounces=8, steps=8, blur=0.0)
    o.reset(mvp, seeds[0])
    o.render(mvp, seeds[1])
    assert _same(ph, o.photons).all()
    assert (ph[:, 8] == 0xFFFFFFFF).any() or (ph[:, 7] > 0).any()


def test_fma32_exhaustive_ties():
    """fma32's tie handling against exact rational arithmetic on constructed
    midpoint cases (a*b + c exactly halfway between two f32, nudged by c)."""
    import subprocess
    from fractions import Fraction
    rng = np.random.default_rng(5)
    cases = []
    for _ in range(400):
        a = np.float32(rng.uniform(1, 2))
        b = np.float32(rng.uniform(1, 2))
        c = np.float32(rng.choice([-1, 1]) * rng.uniform(0, 4) * 2.0 ** rng.integers(-30, 3))
        cases.append((a, b, c))
    # products whose exact value sits on an f32 midpoint: (1 + 2^-12)^2 etc.
    for k in range(1, 12):
        a = np.float32(1 + 2.0 ** -k)
        cases.append((a, a, np.float32(0)))
        cases.append((a, a, np.float32(2.0 ** -40)))
        cases.append((a, a, np.float32(-(2.0 ** -40))))
    arr = np.array(cases, np.float32)
    src = ("const {fma32}=require(process.argv[1]);const a=JSON.parse(require('fs')"
           ".readFileSync(0,'utf8'));const o=new Float32Array(a.length);"
           "for(let i=0;i<a.length;i++)o[i]=fma32(a[i][0],a[i][1],a[i][2]);"
           "process.stdout.write(JSON.stringify(Array.from(new Uint32Array(o.buffer))));")
    out = subprocess.run([js_march.node(), "-e", src, str(js_march.HERE / "mcm_march.js")],
                         input=__import__("json").dumps(arr.astype(float).tolist()),
                         capture_output=True, text=True, check=True)
    got = np.array(__import__("json").loads(out.stdout), np.uint32)
    for (a, b, c), g in zip(arr, got):
        exact = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
        want = np.float32(_round_f32(exact))
        assert want.view(np.uint32) == g, (a, b, c)


def _round_f32(q):
    """Correctly rounded (nearest, ties to even) f32 of a rational."""
    from fractions import Fraction
    if q == 0:
        return 0.0
    x = np.float32(float(q))  # within an ulp; fix up by exact comparison
    cands = [np.nextafter(x, np.float32(-np.inf)), x, np.nextafter(x, np.float32(np.inf))]
    best = min(cands, key=lambda v: (abs(Fraction(float(v)) - q),
                                     int(np.float32(v).view(np.uint32)) & 1))
    return float(best)


@pytest.mark.parametrize("fn", [0, 1, 2])
def test_js_primitives_match_c_oracle(fn, tmp_path):
    """log (fn 0) on a strided sweep of (0, 1] plus specials, sin/cos (fn 1, 2)
    on [0, 2pi] + margin: the JS primitives equal mcm_oracle.c's bit for bit."""
    import subprocess
    if fn == 0:
        u = np.concatenate([np.arange(0, 0x3F800001, 997, dtype=np.uint32),
                            np.array([0x7F800000, 0x80000000, 0xFF800000, 0x7FC00000, 1, 0x7F7FFFFF],
                                     np.uint32)])
    else:
        u = np.linspace(-0.1, 6.4, 400001, dtype=np.float32).view(np.uint32)
    u.tofile(tmp_path / "in.bin")
    expr = ["M.specLog(f[i])", "(M.specSinCos(f[i]), M.sc[0])", "(M.specSinCos(f[i]), M.sc[1])"][fn]
    src = (f"const M=require({str(js_march.HERE / 'mcm_march.js')!r});const fs=require('fs');"
           f"const b=fs.readFileSync({str(tmp_path / 'in.bin')!r});"
           "const f=new Float32Array(b.buffer,b.byteOffset,b.length/4);const o=new Float32Array(f.length);"
           f"for(let i=0;i<f.length;i++)o[i]={expr};"
           f"fs.writeFileSync({str(tmp_path / 'out.bin')!r},Buffer.from(o.buffer));")
    subprocess.run([js_march.node(), "-e", src], check=True, timeout=300)
    got = np.fromfile(tmp_path / "out.bin", np.uint32)
    want = orc.Oracle(4).eval_batch(fn, u)
    assert _same(got, want).all(), f"fn {fn}: {int((~_same(got, want)).sum())} differ"
