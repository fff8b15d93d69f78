"""Statistical parity: the converged image does not depend on the
arithmetic choices the WGSL specification leaves open.

The bit-exact tests pin the HIP march to one arithmetic specification
(fused products, a/b = a*RN(1/b), polynomial log/sin/cos). A
WebGPU implementation may legally use another: libm-accurate transcendentals,
true division, no fusion (oracle liboracle_alt.so, -DORC_ALT). Photon paths then
decorrelate after the first decision flip, so the two are compared as
estimators: K independent replicas of P progressive passes each, per pixel and
channel a Welch z-score of the replica means of the fp32 radiance_to_rgb image
(wgsl:304-326), and a Welch t of the replica frame means per channel (all
pixels pooled). Unbiased arithmetic gives z ~ N(0, 1): max |z| below 6, mean
z^2 near 1, |t_frame| below 4.5. A negative control (the same estimator with a
25 % extinction bias) must fail those bounds: measured t_frame 6-11 and mean
z^2 1.26 (an 8 % bias gives t_frame up to 3.3: below this test's resolution).
"""
import numpy as np
import pytest

import oracle as orc
from vptmcm import configs as cf

K, P = 32, 32  # replicas, passes per replica


def _replica_images(make, R, K, P, rank0):
    """[K, R, R, 3] fp32 images: replica k = reset + P passes on rank seed stream rank0 + k."""
    out = np.empty((K, R, R, 3), np.float32)
    for k in range(K):
        seeds = cf.seed_stream(P + 1, start=0, rank=rank0 + k)
        out[k] = make(seeds)
    return out


def _z(a, b):
    """Welch z per pixel-channel; entries where both estimators are constant
    (e.g. a channel that is exactly 0 in every replica) must agree exactly and
    are left out of the statistics."""
    ma, mb = a.mean(0, dtype=np.float64), b.mean(0, dtype=np.float64)
    va, vb = a.var(0, ddof=1, dtype=np.float64), b.var(0, ddof=1, dtype=np.float64)
    den = np.sqrt(va / a.shape[0] + vb / b.shape[0])
    same = den == 0
    assert (ma[same] == mb[same]).all(), "zero-variance pixels with different means"
    assert (~same).mean() > 0.5, "too few pixels with variance to test"
    return ((ma - mb) / np.where(same, 1.0, den))[~same]


def _frame_t(a, b):
    """Welch t per channel of the replica frame means (all pixels pooled): the
    statistic with the power to see a global bias."""
    fa = a.reshape(a.shape[0], -1, 3).mean(1, dtype=np.float64)
    fb = b.reshape(b.shape[0], -1, 3).mean(1, dtype=np.float64)
    return (fa.mean(0) - fb.mean(0)) / np.sqrt(fa.var(0, ddof=1) / len(fa) + fb.var(0, ddof=1) / len(fb))


def _biased(a, b):
    z, t = _z(a, b), _frame_t(a, b)
    return {"max|z|": float(np.abs(z).max()), "mean z^2": float((z ** 2).mean()),
            "max|t_frame|": float(np.abs(t).max())}


def _assert_unbiased(a, b, what):
    st = _biased(a, b)
    assert st["max|z|"] < 6.0, f"{what}: {st}"
    assert 0.85 < st["mean z^2"] < 1.18, f"{what}: {st}"
    assert st["max|t_frame|"] < 4.5, f"{what}: {st}"


def _oracle_maker(R, vol, tf, ext, alt, mvp, spec="12"):
    spd, ld = cf.light_default()

    def make(seeds):
        o = orc.Oracle(R, alt=alt)
        o.set_spectrum(cf.spectrum_buffer(spec))
        o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
        o.params.update(extinction=ext, bounces=8, steps=8)
        o.reset(mvp, seeds[0], nthreads=8)
        for s in seeds[1:]:
            rgb, _ = o.render(mvp, s, nthreads=8)
        return rgb
    return make


def test_spec_vs_alternative_arithmetic_cpu():
    """C oracle (spec) against the alternative-arithmetic oracle on a 32^3 fBm
    volume, spectral TF (HG g = 0.70), R = 32: statistically identical; the
    negative control (extinction 16 vs 20) is detected."""
    R, vol, tf, mvp = 32, cf.fbm_volume(32, 77, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    a = _replica_images(_oracle_maker(R, vol, tf, 16.0, False, mvp), R, K, P, 1)
    b = _replica_images(_oracle_maker(R, vol, tf, 16.0, True, mvp), R, K, P, 1001)
    _assert_unbiased(a, b, "spec vs alt")
    # negative control: the same estimator with a 25 % extinction bias (what a
    # badly biased distance sampler would do) must be flagged
    c = _replica_images(_oracle_maker(R, vol, tf, 20.0, True, mvp), R, K, P, 2001)
    st = _biased(a, c)
    assert st["max|t_frame|"] >= 4.5 or st["mean z^2"] >= 1.18 or st["max|z|"] >= 6.0, \
        f"negative control not detected: {st}"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["C1_sphere", "C3_fbm"])
def test_gpu_vs_alternative_arithmetic(case):
    """The HIP march (the spec arithmetic, bit-exact with the C oracle) against
    the alternative-arithmetic oracle: C1-like (64^3 sphere, ext 1) and C3-like
    (64^3 fBm, spectral TF, ext 32) at R = 64, K = 32 replicas x P = 32 passes."""
    import vptmcm
    R, mvp = 64, cf.default_mvp_inverse()
    if case == "C1_sphere":
        vol, tf, ext = cf.sphere_in_cube(64), cf.tf_spectral(), 1.0
    else:
        vol, tf, ext = cf.fbm_volume(64, 512, nthreads=8), cf.tf_spectral(), 32.0
    spd, ld = cf.light_default()
    gpu = vptmcm.Renderer(R, device=0)
    gpu.set_spectrum(cf.spectrum_buffer("12"))
    gpu.set_volume(vol)
    gpu.set_material_tf(tf)
    gpu.set_light(spd, ld)
    gpu.set_params(extinction=ext, bounces=8, steps=8)

    def make_gpu(seeds):
        gpu.reset(mvp, seeds[0])
        gpu.render_passes(mvp, seeds[1:])
        return gpu.read_rgb()

    a = _replica_images(make_gpu, R, K, P, 1)
    gpu.close()
    b = _replica_images(_oracle_maker(R, vol, tf, ext, True, mvp), R, K, P, 1001)
    _assert_unbiased(a, b, f"{case}: HIP vs alt")


@pytest.mark.gpu
def test_gpu_vs_alternative_arithmetic_c3_full_size():
    """The headline configuration itself (BASELINE C3: 512^3 fBm, spectral TF,
    R = 512, S = 8, extinction 32, default camera): the HIP march against the
    alternative-arithmetic oracle, K = 32 replicas x P = 32 passes each
    (2.1 G photon-steps of CPU oracle). The statistics must show no bias, and
    the test proves its own resolution: a 2 % multiplicative bias of the
    alternative images, and a 3 % extinction bias of the HIP march itself, must
    both be flagged (frame-mean t over 262,144 pixels per replica)."""
    import vptmcm
    R, mvp, ext = 512, cf.default_mvp_inverse(), 32.0
    vol, tf = cf.fbm_volume(512, 512, nthreads=cf.host_threads()), cf.tf_spectral()
    spd, ld = cf.light_default()
    gpu = vptmcm.Renderer(R, device=0)
    gpu.set_spectrum(cf.spectrum_buffer("12"))
    gpu.set_volume(vol)
    gpu.set_material_tf(tf)
    gpu.set_light(spd, ld)

    def make_gpu(e):
        def make(seeds):
            gpu.set_params(extinction=e, bounces=8, steps=8)
            gpu.reset(mvp, seeds[0])
            gpu.render_passes(mvp, seeds[1:])
            return gpu.read_rgb()
        return make

    a = _replica_images(make_gpu(ext), R, K, P, 1)
    c = _replica_images(make_gpu(ext * 1.03), R, K, P, 3001)
    gpu.close()
    nt = cf.host_threads()
    spec = cf.spectrum_buffer("12")

    def make_alt(seeds):
        o = orc.Oracle(R, alt=True)
        o.set_spectrum(spec)
        o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
        o.params.update(extinction=ext, bounces=8, steps=8)
        o.reset(mvp, seeds[0], nthreads=nt)
        for s in seeds[1:]:
            rgb, _ = o.render(mvp, s, nthreads=nt)
        return rgb

    b = _replica_images(make_alt, R, K, P, 1001)
    _assert_unbiased(a, b, "C3 full size: HIP vs alt")
    for what, biased in (("2 % image bias", (b * np.float32(1.02))), ("3 % extinction bias", c)):
        st = _biased(a, biased)
        assert st["max|t_frame|"] >= 4.5 or st["mean z^2"] >= 1.18 or st["max|z|"] >= 6.0, \
            f"C3 negative control ({what}) not detected: {st}"
