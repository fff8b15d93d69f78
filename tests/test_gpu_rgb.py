"""The RGB sibling renderer ('mcm-compute', MCMComputeRenderer.wgsl)
through the C-ABI against its CPU oracle: bit-exact photon state (64-B Photon)
and rgba16float image, same arithmetic specification as the spectral path."""
import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf

pytestmark = pytest.mark.gpu


def tf_rgb(kind: str) -> np.ndarray:
    x = np.arange(256)
    if kind == "default":
        return np.array([[[255, 0, 0, 0], [255, 0, 0, 255]]], np.uint8)
    if kind == "ramp":  # alpha ramp, warm-to-cool colour, 256 x 1
        t = np.zeros((1, 256, 4), np.uint8)
        t[0, :, 0] = 255 - x // 2
        t[0, :, 1] = 128 + x // 4
        t[0, :, 2] = x
        t[0, :, 3] = np.clip((x - 40) * 2, 0, 255)
        return t
    t = np.zeros((7, 100, 4), np.uint8)  # odd size, several rows (only row 0 is sampled)
    t[..., 0] = 200
    t[..., 1] = np.arange(100)[None, :] * 2
    t[..., 2] = 90
    t[..., 3] = 255 - np.arange(100)[None, :]
    return t


def same_words(a, b):
    fa, fb = a.view(np.float32), b.view(np.float32)
    return (a == b) | (np.isnan(fa) & np.isnan(fb))


@pytest.mark.parametrize("layout", [vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_LINEAR, vptmcm.LAYOUT_BRICK8,
                                    vptmcm.LAYOUT_COLUMN4])
@pytest.mark.parametrize("tfk,aniso,ext,env", [("default", 0.0, 1.0, (255, 255, 255, 255)),
                                               ("ramp", 0.6, 24.0, (255, 255, 255, 255)),
                                               ("odd", -0.4, 8.0, (200, 150, 90, 255)),
                                               ("ramp", 0.0, 32.0, (255, 255, 255, 255))])
@pytest.mark.parametrize("maj", ["auto", "on"])
def test_rgb_renderer_bitexact(layout, tfk, aniso, ext, env, maj, monkeypatch):
    """maj: VPTMCM_MAJ (on: every launch with the macro-cell alpha bound,
    except on LINEAR, which keeps no macro table)."""
    monkeypatch.setenv("VPTMCM_MAJ", maj)
    R = 64
    vol = cf.fbm_volume(48, 13)
    gpu = vptmcm.Renderer(R, device=0, layout=layout, renderer=vptmcm.RENDERER_RGB)
    cpu = orc.OracleRGB(R)
    tf = tf_rgb(tfk)
    if tfk != "default":
        gpu.set_transfer_function(tf)
    gpu.set_environment(env)
    gpu.set_volume(vol)
    gpu.set_params(extinction=ext, anisotropy=aniso, bounces=8, steps=8)
    cpu.volume, cpu.tf, cpu.env = vol, tf, np.array(env, np.uint8)
    cpu.params.update(extinction=ext, anisotropy=aniso, bounces=8, steps=8)
    mvp = cf.golden_mvp("orbit") if tfk == "odd" else cf.default_mvp_inverse()
    seeds = cf.seed_stream(6, start=40)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0])
    assert same_words(gpu.read_photons(), cpu.photons).all(), "reset"
    for k, s in enumerate(seeds[1:4], 1):
        gpu.render(mvp, s)
        _, want = cpu.render(mvp, s)
        ok = same_words(gpu.read_photons(), cpu.photons)
        assert ok.all(), f"pass {k}: {int((~ok).sum())} photon words differ"
        assert np.array_equal(gpu.read_rgba16f(), want), f"pass {k}: image differs"
    gpu.render_passes(mvp, seeds[4:])  # fused launch
    for s in seeds[4:]:
        _, want = cpu.render(mvp, s)
    assert same_words(gpu.read_photons(), cpu.photons).all(), "fused"
    assert np.array_equal(gpu.read_rgba16f(), want)
    if maj == "on":
        assert gpu.last_launch()["macro"] == (layout != vptmcm.LAYOUT_LINEAR)
    gpu.close()


def test_rgb_environment_and_tf_validation():
    g = vptmcm.Renderer(16, device=0, renderer=vptmcm.RENDERER_RGB)
    env4 = np.zeros(16, np.uint8)
    with pytest.raises(vptmcm.VptError, match="1x1"):
        g._ck(g.L.vptmcm_set_environment(g.h, env4.ctypes.data, 2, 2))
    with pytest.raises(vptmcm.VptError):
        g.set_transfer_function(np.zeros((1, 5000, 4), np.uint8))
    s = vptmcm.Renderer(16, device=0)
    with pytest.raises(vptmcm.VptError):
        s.set_transfer_function(np.zeros((1, 4, 4), np.uint8))
    g.close()
    s.close()


@pytest.mark.parametrize("camera,maj", [("default", "auto"), ("near", "auto"), ("orbit_tilted", "auto"),
                                        ("near", "on"), ("default", "on")])
def test_rgb_fused_schedule_robust(camera, maj, monkeypatch):
    """Fused multi-pass launches of the RGB march at R = 128: the tile schedule
    (volume flags carried between launches), the volume-wave priority, the
    robust-miss path (start points materialised at the end of the launch) and
    the FAST geometry, bit-exact against the oracle after every launch; with
    the macro-cell alpha bound pinned on as well."""
    monkeypatch.setenv("VPTMCM_MAJ", maj)
    R = 128
    vol = cf.fbm_volume(64, 21)
    gpu = vptmcm.Renderer(R, device=0, renderer=vptmcm.RENDERER_RGB)
    cpu = orc.OracleRGB(R)
    tf = tf_rgb("ramp")
    gpu.set_transfer_function(tf)
    gpu.set_environment((255, 230, 200, 255))
    gpu.set_volume(vol)
    gpu.set_params(extinction=24.0, anisotropy=0.7, bounces=8, steps=8)
    cpu.volume, cpu.tf, cpu.env = vol, tf, np.array((255, 230, 200, 255), np.uint8)
    cpu.params.update(extinction=24.0, anisotropy=0.7, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse() if camera == "default" else cf.golden_mvp(camera)
    seeds = cf.seed_stream(13, start=70)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0])
    for launch in range(3):
        ss = seeds[1 + 4 * launch:5 + 4 * launch]
        gpu.render_passes(mvp, ss)
        for s in ss:
            _, want = cpu.render(mvp, s)
        ok = same_words(gpu.read_photons(), cpu.photons)
        assert ok.all(), f"{camera} launch {launch}: {int((~ok).sum())} photon words differ"
        assert np.array_equal(gpu.read_rgba16f(), want), f"{camera} launch {launch}: image"
    gpu.close()
