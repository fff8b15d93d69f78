"""Exhaustive proofs, on the GPU, that the fast arithmetic sequences the march
kernels use are bit-identical to the correctly rounded IEEE results the
arithmetic specification (and the CPU oracle) prescribe.

Each check evaluates the exact device function used by the kernels on every
u32 bit pattern of its domain (2^32 inputs for rcp and sqrt) and compares it
with hipcc's IEEE division / sqrt (NaN == NaN)."""
import pytest

import vptmcm

pytestmark = pytest.mark.gpu

ALL = (0, 1 << 32)


@pytest.mark.parametrize("fn,name,lo,n", [
    (6, "rcp_cr: RN(1/x)", *ALL),
    (7, "sqrt_cr: RN(sqrt x)", *ALL),
    (8, "log_div: RN(f/(2+f)) on m in [sqrt(.5), sqrt(2)]", 0x3F3504F3, 0x3FB504F4 - 0x3F3504F3),
    (9, "spec_log_unit(h) == spec_log(f32(h) * 2^-32)", *ALL),
    (10, "rcp_small: RN(1/x) for finite |x| < 2^126 and NaN", *ALL),
    (11, "sqrt_z: RN(sqrt x) for +-0, NaN, normal x < 0, x > 0 with exponent 32..254", *ALL),
    (12, "rcp_in_range: RN(1/x) for exponent 1..252", *ALL),
    (15, "clampc_q (v_max/v_min) == clampc for non-signalling x", *ALL),
    (16, "v_min/v_max/v_max3 == smin/smax chains (quiet, no +-0 pair)", *ALL),
    (17, "inv_len: RN(1/RN(sqrt x)) with one guard", *ALL),
])
def test_fast_sequences_are_correctly_rounded(fn, name, lo, n):
    with vptmcm.Renderer(8, device=0) as g:
        bad, first = g.debug_verify(fn, lo, n, 8)
    assert bad == 0, f"{name}: {bad} mismatches, e.g. {[hex(int(v)) for v in first]}"


def test_unguarded_estimates_are_not_exact():
    """Sanity check of the checker: the raw hardware estimates are NOT correctly
    rounded, so the guards/corrections above are doing real work."""
    with vptmcm.Renderer(8, device=0) as g:
        assert g.debug_verify(0, *ALL, 0)[0] > 0   # raw v_rcp_f32
        assert g.debug_verify(2, *ALL, 0)[0] > 0   # raw v_sqrt_f32
        assert g.debug_verify(1, *ALL, 0)[0] > 0   # rcp + Newton without the range guard


@pytest.mark.parametrize("layout", ["12", "uniform6", "shifted", "narrow"])
def test_arithmetic_bin_search_matches_sequential(layout):
    """bin_of's arithmetic path (equal-width bins) equals the reference's
    first-match search (wgsl:276-290) for the wavelength of every h5."""
    import numpy as np
    from vptmcm import configs as cf
    bufs = {"12": cf.spectrum_buffer("12")}
    def uniform(nb, lam0, w):
        b = np.zeros(64, np.float32)
        b[0] = nb
        b[1:nb + 2] = [np.float32(lam0) + np.float32(i) * np.float32(w) for i in range(nb + 1)]
        return b
    bufs["uniform6"] = uniform(6, 400.0, 50.0)
    bufs["shifted"] = uniform(12, 380.75, 26.25)
    bufs["narrow"] = uniform(12, 500.0, 0.75)
    with vptmcm.Renderer(8, device=0) as g:
        g.set_spectrum(bufs[layout])
        assert g.uniform_bins(), "host did not take the arithmetic path for equal-width bins"
        bad, first = g.debug_verify(13, *ALL, 8)
    assert bad == 0, f"{layout}: {bad} mismatching h5, e.g. {[hex(int(v)) for v in first]}"
