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
