"""Every environment knob the library reads ("Environment
knobs") leaves every result bit unchanged: the same small
case — a fused call, queued render() passes, a camera change, timing on — is
rendered once per knob setting, each in a fresh handle (knobs are read at
vptmcm_create), and photons, the fp32 image and the rgba16f image must equal
the knob-free run, which itself equals the oracle."""
import numpy as np
import pytest

import vptmcm
from vptmcm import configs as cf

from test_gpu_parity import assert_photons_equal, assert_rgb32_equal, assert_rgba_equal, make_pair

pytestmark = pytest.mark.gpu

# (variable, value): every documented knob, each variant bit of VPTMCM_MARCH_VARIANT
KNOBS = [("VPTMCM_MARCH_VARIANT", str(b)) for b in (1, 2, 4, 8, 16, 32, 64, 128, 256)] + [
    ("VPTMCM_MARCH_VARIANT", "511"),
    ("VPTMCM_MAJ", "on"),
    ("VPTMCM_MAJ", "off"),
    ("VPTMCM_DARK", "0"),
    ("VPTMCM_DONE_FLAG", "0"),
    ("VPTMCM_SCHED_CACHE", "0"),
    ("VPTMCM_TIME_STOP", "0"),
    ("VPTMCM_TIME_BEGIN", "marker"),
    ("VPTMCM_SYNC_SPIN_US", "0"),
    ("VPTMCM_SYNC_SPIN", "1"),
    ("VPTMCM_COMM_TRACE", "1"),
    ("VPTMCM_COMM_TIMEOUT_MS", "5000"),
]


def _run(layout, tf, spec, with_oracle=False, devices=None):
    R = 64
    vol = cf.fbm_volume(48, 21, nthreads=8)
    gpu, cpu = make_pair(R, vol, tf, spec=spec, ext=24.0, layout=layout)
    if devices is not None:  # the same inputs behind a device-list handle
        gpu.close()
        gpu = vptmcm.Renderer(R, layout=layout, devices=devices)
        gpu.set_spectrum(cf.spectrum_buffer(spec))
        gpu.set_volume(vol)
        gpu.set_material_tf(tf)
        gpu.set_light(cpu.light, cpu.light_dir)
        gpu.set_params(extinction=24.0, bounces=8, steps=8)
    m1, m2 = cf.golden_mvp("orbit"), cf.default_mvp_inverse()
    seeds = cf.seed_stream(14, start=3)
    gpu.enable_kernel_timing(True)
    gpu.reset(m1, seeds[0])
    gpu.render_passes(m1, seeds[1:7])
    for s in seeds[7:10]:
        gpu.render(m1, s)
    for s in seeds[10:]:
        gpu.render(m2, s)
    gpu.synchronize()
    ms, n = gpu.kernel_time()
    assert n >= 2 and ms > 0
    got = (gpu.read_photons(), gpu.read_rgb(), gpu.read_rgba16f(), gpu.last_launch()["macro"])
    gpu.close()
    if with_oracle:
        cpu.reset(m1, seeds[0], nthreads=16)
        for k, s in enumerate(seeds[1:], 1):
            rgb, want = cpu.render(m1 if k < 10 else m2, s, nthreads=16)
        assert_photons_equal(got[0], cpu.photons, "no knobs vs oracle")
        assert_rgb32_equal(got[1], rgb, "no knobs vs oracle")
        assert_rgba_equal(got[2], want, "no knobs vs oracle")
    return got


@pytest.mark.parametrize("layout,tfname,spec", [(vptmcm.LAYOUT_COLUMN4, "spectral", "12"),
                                                (vptmcm.LAYOUT_CORNER8, "spectral", "12"),
                                                (vptmcm.LAYOUT_BRICK8, "materials", "8_uneven")])
def test_every_knob_leaves_the_bits(layout, tfname, spec, monkeypatch):
    tf = cf.tf_spectral() if tfname == "spectral" else cf.tf_materials(True)
    for var, _ in KNOBS:
        monkeypatch.delenv(var, raising=False)
    base = _run(layout, tf, spec, with_oracle=True)
    for var, val in KNOBS:
        monkeypatch.setenv(var, val)
        got = _run(layout, tf, spec)
        monkeypatch.delenv(var)
        what = f"{var}={val}"
        if var == "VPTMCM_MAJ":  # the last launch ran k_march<..., MAJ> as asked
            assert got[3] == (val == "on"), what
        assert_photons_equal(got[0], base[0], what)
        assert_rgb32_equal(got[1], base[1], what)
        assert_rgba_equal(got[2], base[2], what)


def test_every_knob_leaves_the_bits_device_list(monkeypatch):
    """The same sweep on a device-list handle of three replicas (device 0
    repeated; the default COLUMN4 layout and PEER transport), with
    VPTMCM_GROUP_THREADS=0 (serial forwarding) among the knobs: replica 0's
    photons, the composite's fp32 and rgba16f images equal the knob-free run's.
    Replica 0's photons also equal the single-device handle's (the knob-free
    single run is pinned to the oracle above)."""
    tf = cf.tf_spectral()
    knobs = KNOBS + [("VPTMCM_GROUP_THREADS", "0")]
    for var, _ in knobs:
        monkeypatch.delenv(var, raising=False)
    single = _run(vptmcm.LAYOUT_COLUMN4, tf, "12", with_oracle=True)
    base = _run(vptmcm.LAYOUT_COLUMN4, tf, "12", devices=[0, 0, 0])
    assert_photons_equal(base[0], single[0], "device list replica 0 vs single handle")
    assert not np.array_equal(base[2], single[2])  # the target is the 3-replica composite
    for var, val in knobs:
        monkeypatch.setenv(var, val)
        got = _run(vptmcm.LAYOUT_COLUMN4, tf, "12", devices=[0, 0, 0])
        monkeypatch.delenv(var)
        what = f"device list, {var}={val}"
        assert_photons_equal(got[0], base[0], what)
        assert_rgb32_equal(got[1], base[1], what)
        assert_rgba_equal(got[2], base[2], what)


def test_auto_bound_follows_the_measurement(monkeypatch):
    """VPTMCM_MAJ=auto (the default) times pairs of launches with and without
    the macro-cell alpha bound outside timed regions and keeps the faster: at
    the near camera on C3's 512^3 volume the bound saves ~26 % of a pass
    (profiles/r06/s18), far beyond the pairs' spread, so after a dozen
    32-pass launches read back by synchronize the march runs with it. A camera
    that then moves every launch (an interactive rotation) never completes a
    pair of launches, so the decision stands."""
    for var in ("VPTMCM_MAJ", "VPTMCM_MARCH_VARIANT"):
        monkeypatch.delenv(var, raising=False)
    vol = cf.fbm_volume(512, 512, nthreads=8)
    gpu = vptmcm.Renderer(512, device=0, layout=vptmcm.LAYOUT_COLUMN4)
    gpu.set_spectrum(cf.spectrum_buffer("12"))
    gpu.set_volume(vol)
    gpu.set_material_tf(cf.tf_spectral())
    gpu.set_light(np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32))
    gpu.set_params(extinction=32.0, bounces=8, steps=8)
    mn = cf.golden_mvp("near")
    seeds = cf.seed_stream(1 + 12 * 32, start=5)
    gpu.reset(mn, seeds[0])
    for j in range(12):
        gpu.render_passes(mn, seeds[1 + 32 * j: 1 + 32 * (j + 1)])
        gpu.synchronize()
    info = gpu.last_launch()
    assert info["macro"] and info["passes"] == 32, info
    rseeds = cf.seed_stream(8 * 32, start=900)
    for j in range(8):  # a new matrix every launch
        m = mn.copy()
        m[12] += np.float32(1e-4 * (j + 1))
        gpu.render_passes(m, rseeds[32 * j: 32 * (j + 1)])
        gpu.synchronize()
        assert gpu.last_launch()["macro"], j
    gpu.close()


@pytest.mark.parametrize("layout", [vptmcm.LAYOUT_COLUMN4, vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_BRICK8])
def test_macro_bound_empty_space_bitexact(layout, monkeypatch):
    """The reference's two-spheres test volume (generate_test_volume.ipynb):
    mostly empty space, whose macro cells carry alpha code 0 (every wheel from
    2^-16 up skips the gather there), beside the spheres' cells. Spectral and
    RGB renderers with the bound pinned on, bit-exact against their oracles."""
    import oracle as orc
    from test_gpu_rgb import same_words, tf_rgb
    monkeypatch.setenv("VPTMCM_MAJ", "on")
    vol = cf.two_spheres(48)
    gpu, cpu = make_pair(64, vol, cf.tf_spectral(), ext=24.0, layout=layout)
    mvp, seeds = cf.golden_mvp("orbit"), cf.seed_stream(10, start=21)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:6])
    for s in seeds[1:6]:
        rgb, want = cpu.render(mvp, s, nthreads=16)
    assert gpu.last_launch()["macro"]
    assert_photons_equal(gpu.read_photons(), cpu.photons, "two spheres, bound on")
    assert_rgb32_equal(gpu.read_rgb(), rgb, "two spheres, bound on")
    assert_rgba_equal(gpu.read_rgba16f(), want, "two spheres, bound on")
    gpu.close()
    g = vptmcm.Renderer(64, device=0, layout=layout, renderer=vptmcm.RENDERER_RGB)
    c = orc.OracleRGB(64)
    tf = tf_rgb("ramp")
    g.set_transfer_function(tf)
    g.set_environment((255, 255, 255, 255))
    g.set_volume(vol)
    g.set_params(extinction=24.0, anisotropy=0.6, bounces=8, steps=8)
    c.volume, c.tf, c.env = vol, tf, np.array((255, 255, 255, 255), np.uint8)
    c.params.update(extinction=24.0, anisotropy=0.6, bounces=8, steps=8)
    g.reset(mvp, seeds[0])
    c.reset(mvp, seeds[0])
    g.render_passes(mvp, seeds[1:6])
    for s in seeds[1:6]:
        _, want = c.render(mvp, s)
    assert g.last_launch()["macro"]
    assert same_words(g.read_photons(), c.photons).all(), "rgb two spheres, bound on"
    assert np.array_equal(g.read_rgba16f(), want)
    g.close()


def test_set_macro_skip_modes(monkeypatch):
    """vptmcm_set_macro_skip switches the bound per handle (the env knob only
    sets the initial mode): off / on run k_march<..., MAJ> as asked, the bits
    equal the oracle's either way, a bad mode is refused."""
    monkeypatch.delenv("VPTMCM_MAJ", raising=False)
    gpu, cpu = make_pair(64, cf.fbm_volume(48, 21, nthreads=8), cf.tf_spectral(), ext=24.0,
                         layout=vptmcm.LAYOUT_COLUMN4)
    mvp, seeds = cf.golden_mvp("near"), cf.seed_stream(7, start=33)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    for k, mode in enumerate(["off", "on", "off", "on", "auto", "on"]):
        gpu.set_macro_skip(mode)
        gpu.render_passes(mvp, seeds[1 + k:2 + k])
        rgb, want = cpu.render(mvp, seeds[1 + k], nthreads=16)
        if mode != "auto":
            assert gpu.last_launch()["macro"] == (mode == "on"), mode
    assert_photons_equal(gpu.read_photons(), cpu.photons, "set_macro_skip")
    assert_rgba_equal(gpu.read_rgba16f(), want, "set_macro_skip")
    with pytest.raises(vptmcm.VptError, match="set_macro_skip"):
        gpu._ck(gpu.L.vptmcm_set_macro_skip(gpu.h, 3))
    gpu.close()
