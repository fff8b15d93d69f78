"""The artistic tone mapper (ArtisticToneMapper.wgsl:38-48) on the GPU against the
double-precision oracle, on the renderer's own rgba16float output.

Floating-point bar (stated tolerance): the device evaluates the shader in f32
with the hardware log2/exp2 (pow = exp2(e * log2 x), as WGSL defines it), the
oracle in f64; rgba8 channels may differ by at most 1 LSB where the value lands
within f32 rounding of a quantisation boundary, and >= 99.5 % must be equal."""
import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf

pytestmark = pytest.mark.gpu

PARAMS = [
    dict(),                                                   # the reference defaults
    dict(low=0.0, high=1.0, mid=0.5, saturation=1.0, gamma=1.0),
    dict(low=0.05, high=0.6, mid=0.2, saturation=1.5, gamma=2.2),
    dict(low=-0.1, high=2.0, mid=0.9, saturation=0.0, gamma=1.8),
    dict(low=0.0, high=0.25, mid=0.00001, saturation=3.0, gamma=0.5),
]


@pytest.fixture(scope="module")
def frame():
    g = vptmcm.Renderer(256, device=0)
    g.set_spectrum(cf.spectrum_buffer("12"))
    g.set_volume(cf.fbm_volume(64, 3))
    g.set_material_tf(cf.tf_spectral())
    g.set_light(*cf.light_default())
    g.set_params(extinction=16.0)
    mvp = cf.default_mvp_inverse()
    g.reset(mvp, cf.seed_bits(0))
    g.render_passes(mvp, cf.seed_stream(6))
    yield g
    g.close()


@pytest.mark.parametrize("k", range(len(PARAMS)))
def test_tonemap_matches_oracle(frame, k):
    p = PARAMS[k]
    got = frame.tonemap_artistic(**p)
    want = orc.Oracle(1).tonemap_artistic(frame.read_rgba16f(), **p)
    d = np.abs(got.astype(int) - want.astype(int))
    assert (got[..., 3] == 255).all()
    assert d.max() <= 1, f"params {p}: max diff {d.max()}"
    assert (d == 0).mean() >= 0.995, f"params {p}: only {(d == 0).mean():.4f} equal"
