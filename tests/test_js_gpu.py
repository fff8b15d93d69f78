"""The JavaScript renderer (N-API -> C-ABI -> HIP) against the CPU oracle.

Node drives MCMSpectralComputeRenderer as the reference application drives
WebGPUMCMSpectralComputeRenderer: construct, set the TF, load the volume
through RAWReader/Volume (which resets: first reset sees the all-zero spectrum
buffer, as in the reference), render K passes with Math.random()-style seeds.
The oracle replays the same call sequence; photons and image must be bit-exact.
"""
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle as orc
from vptmcm import configs as cf

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def run_case(tmp_path, vol, tf, R=64, passes=3, ext=32.0, layout="corner8", stream=True,
             change_event=False, tonemap=None, bvp=None, ui=None, band=None, render_passes=False,
             devices=None):
    D, H, W = vol.shape
    (tmp_path / "vol.raw").write_bytes(np.ascontiguousarray(vol).tobytes())
    (tmp_path / "tf.bin").write_bytes(np.ascontiguousarray(tf).tobytes())
    seeds = [float(np.uint32(cf.seed_bits(k)).view(np.float32)) for k in range(passes + 6)]
    case = dict(R=R, passes=passes, extinction=ext, bounces=8, steps=8, layout=layout,
                W=W, H=H, D=D, volume_path=str(tmp_path / "vol.raw"), tf_path=str(tmp_path / "tf.bin"),
                seeds=seeds, stream_volume=stream, change_event=change_event, tonemap=tonemap,
                bvp_path=None, ui=ui, band=band, render_passes=render_passes, devices=devices)
    if bvp is not None:
        (tmp_path / "vol.bvp").write_bytes(bvp)
        case["bvp_path"] = str(tmp_path / "vol.bvp")
    (tmp_path / "case.json").write_text(json.dumps(case))
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "gpu_render.js"), str(tmp_path / "case.json"),
                        str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    ph = np.frombuffer((tmp_path / "photons.bin").read_bytes(), np.uint32).reshape(R * R, 36)
    rgba = np.frombuffer((tmp_path / "rgba.bin").read_bytes(), np.uint16).reshape(R, R, 4)
    rgb32 = np.frombuffer((tmp_path / "rgb32.bin").read_bytes(), np.float32).reshape(R, R, 3)
    meta = json.loads((tmp_path / "meta.json").read_text())
    used = meta["seeds_used"]
    run_case.rgb32, run_case.meta = rgb32, meta
    return ph, rgba, seeds, used


def oracle_replay(vol, tf, R, seeds, passes, ext, change_event=False):
    o = orc.Oracle(R)
    o.volume, o.tf, o.light = vol, tf, np.full(256, 100, np.uint8)
    o.params.update(extinction=ext, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    bits = lambda s: int(np.float32(s).view(np.uint32))  # noqa: E731
    o.reset(mvp, bits(seeds[0]))                 # spectrum still all zero here
    o.set_spectrum(cf.spectrum_buffer("12"))     # uploaded by the first render
    rgba = None
    for k in range(passes):
        oracle_replay.rgb32, rgba = o.render(mvp, bits(seeds[1 + k]))
    if change_event:
        o.reset(mvp, bits(seeds[1 + passes]))
    return o.photons, rgba


def same(a, b):
    fa, fb = a.view(np.float32), b.view(np.float32)
    return ((a == b) | (np.isnan(fa) & np.isnan(fb))).all()


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
@pytest.mark.parametrize("render_passes", [False, True])
def test_js_render_calls_fuse(tmp_path, render_passes):
    """40 JS render() calls (each re-sending the unchanged uniforms, as the
    reference does every pass) reach the fused march: 2 launches (32 + 8
    passes), bit-exact; renderPasses(40) takes one N-API call to the same."""
    vol, tf = cf.sphere_in_cube(64), cf.tf_spectral()
    ph, rgba, seeds, used = run_case(tmp_path, vol, tf, passes=40, render_passes=render_passes)
    assert used == 41
    meta = run_case.meta
    assert meta["march_launches"] == 2, meta
    assert meta["last_launch"]["passes"] == 8 and meta["last_launch"]["mode"] == 2, meta
    want_ph, want_rgba = oracle_replay(vol, tf, 64, seeds, 40, 32.0)
    assert same(ph[:, :34], want_ph[:, :34])
    assert np.array_equal(rgba, want_rgba)
    assert same(run_case.rgb32.view(np.uint32), oracle_replay.rgb32.view(np.uint32))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
@pytest.mark.parametrize("layout,stream", [("corner8", True), ("linear", False), ("brick8", True),
                                           ("column4", True), ("column4", False)])
def test_js_renderer_bitexact(tmp_path, layout, stream):
    vol, tf = cf.sphere_in_cube(64), cf.tf_spectral()
    ph, rgba, seeds, used = run_case(tmp_path, vol, tf, layout=layout, stream=stream)
    assert used == 4  # one seed per reset/render, like Math.random() in js:231/298
    want_ph, want_rgba = oracle_replay(vol, tf, 64, seeds, 3, 32.0)
    assert same(ph[:, :34], want_ph[:, :34])
    assert np.array_equal(rgba, want_rgba)
    # getRadianceRGB(): the fp32 image before the f16 store (a13)
    assert same(run_case.rgb32.view(np.uint32), oracle_replay.rgb32.view(np.uint32))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_property_change_resets(tmp_path):
    vol, tf = cf.two_spheres(48), cf.tf_materials(True)
    ph, _, seeds, used = run_case(tmp_path, vol, tf, R=48, passes=2, ext=16.0, change_event=True)
    assert used == 4
    want_ph, _ = oracle_replay(vol, tf, 48, seeds, 2, 16.0, change_event=True)
    assert same(ph[:, :34], want_ph[:, :34])
    assert (ph[:, 7] == 0).all()  # samples cleared by the reset


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_tonemapper(tmp_path):
    """ToneMapperFactory('artistic') on the renderer's target, through N-API, against
    the double-precision oracle of ArtisticToneMapper.wgsl (<= 1 LSB, >= 99.5 % equal)."""
    vol, tf = cf.sphere_in_cube(64), cf.tf_spectral()
    tm = dict(low=0.0, high=0.8, mid=0.3, saturation=1.2, gamma=2.2)
    _, rgba, _, _ = run_case(tmp_path, vol, tf, tonemap=tm)
    ldr = np.frombuffer((tmp_path / "ldr.bin").read_bytes(), np.uint8).reshape(64, 64, 4)
    want = orc.Oracle(1).tonemap_artistic(rgba, **tm)
    d = np.abs(ldr.astype(int) - want.astype(int))
    assert d.max() <= 1 and (d == 0).mean() >= 0.995


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_bvp_volume_streams_bitexact(tmp_path):
    """A bricked BVP archive (48 placements, some blocks deflated) streamed
    block by block into HBM (vptmcm_volume_write_block) renders bit-exactly like
    the oracle on the assembled volume."""
    from bvp import write_bvp
    vol, tf = cf.fbm_volume(64, 8), cf.tf_spectral()
    ph, rgba, seeds, _ = run_case(tmp_path, vol, tf, bvp=write_bvp(vol, (16, 32, 24), 5))
    want_ph, want_rgba = oracle_replay(vol, tf, 64, seeds, 3, 32.0)
    assert same(ph[:, :34], want_ph[:, :34])
    assert np.array_equal(rgba, want_rgba)


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_rgb_renderer_bitexact(tmp_path):
    """RendererFactory('mcm-compute') (the RGB sibling, MCMComputeRenderer.wgsl)
    through N-API against the RGB oracle, with a coloured environment texel."""
    from test_gpu_rgb import tf_rgb
    vol, tf = cf.fbm_volume(48, 13), tf_rgb("ramp")
    D, H, W = vol.shape
    (tmp_path / "vol.raw").write_bytes(np.ascontiguousarray(vol).tobytes())
    (tmp_path / "tf.bin").write_bytes(tf.tobytes())
    seeds = [float(np.uint32(cf.seed_bits(k)).view(np.float32)) for k in range(5)]
    env = [230, 200, 170, 255]
    case = dict(R=64, passes=3, extinction=16.0, bounces=8, steps=8, layout="corner8", W=W, H=H, D=D,
                volume_path=str(tmp_path / "vol.raw"), tf_path=str(tmp_path / "tf.bin"), seeds=seeds,
                stream_volume=True, change_event=False, tonemap=None, bvp_path=None,
                renderer="mcm-compute", anisotropy=0.5, tf_w=tf.shape[1], tf_h=tf.shape[0], env=env)
    (tmp_path / "case.json").write_text(json.dumps(case))
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "gpu_render.js"), str(tmp_path / "case.json"),
                        str(tmp_path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    ph = np.frombuffer((tmp_path / "photons.bin").read_bytes(), np.uint32).reshape(64 * 64, 16)
    rgba = np.frombuffer((tmp_path / "rgba.bin").read_bytes(), np.uint16).reshape(64, 64, 4)
    o = orc.OracleRGB(64)
    o.volume, o.tf, o.env = vol, tf, np.array(env, np.uint8)
    o.params.update(extinction=16.0, anisotropy=0.5, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    bits = lambda s: int(np.float32(s).view(np.uint32))  # noqa: E731
    o.reset(mvp, bits(seeds[0]))
    for k in range(3):
        _, want = o.render(mvp, bits(seeds[1 + k]))
    assert same(ph, o.photons)
    assert np.array_equal(rgba, want)


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_ui_models_drive_renderer_bitexact(tmp_path):
    """The headless UI models (js/ui.js: MaterialTransferFunction, SpectrumRepresentation
    with exponential markers, LightEditor) wired to the renderer: every model change resets
    (js:116-125), the first render uploads their spectrum; the materials TF has few distinct
    rows and 8 uneven bins, so the march runs its deduplicated-TF, bin-table MODE 6. Bit-exact vs the
    oracle replaying the same inputs."""
    col = list(range(60, 60 + 256))
    ui = {"materials": [{"albedo": 180, "alpha": 60, "anisotropy": 127, "rows": [20, 89]},
                        {"albedo": 150, "alpha": 140, "anisotropy": 200, "rows": [90, 169]},
                        {"albedo": 230, "alpha": 230, "anisotropy": [min(255, v) for v in col],
                         "rows": [170, 255]}],
          "n_bins": 8, "k": 1.5, "direction": [0.6, 0.8, 0.0]}
    vol = cf.fbm_volume(64, 5, nthreads=8)
    R, passes = 64, 3
    ph, rgba, seeds, used = run_case(tmp_path, vol, cf.tf_zero(), R=R, passes=passes, ui=ui)
    spec = np.frombuffer((tmp_path / "spectrum.bin").read_bytes(), np.float32)
    tf = np.frombuffer((tmp_path / "tf_used.bin").read_bytes(), np.uint8).reshape(256, 256, 4)
    assert int(spec[0] + 0.5) == 8
    o = orc.Oracle(R)
    o.volume, o.tf, o.light = vol, tf, np.full(256, 100, np.uint8)
    o.light_dir = np.array(ui["direction"], np.float32)
    o.params.update(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    bits = lambda s: int(np.float32(s).view(np.uint32))  # noqa: E731
    n_resets = used - passes  # the three model connections and the volume load
    assert n_resets == 4
    o.reset(mvp, bits(seeds[n_resets - 1]))  # a full reset: only the last one is visible
    o.set_spectrum(spec)                     # uploaded by the first render (js:311)
    for k in range(passes):
        _, want = o.render(mvp, bits(seeds[n_resets + k]))
    assert same(ph[:, :34], o.photons[:, :34])
    assert np.array_equal(rgba, want)


def test_js_mode_b_band_matches_full_frame(tmp_path):
    """renderer.setBand (N-API setBand -> vptmcm_set_band): the band rows of photons,
    rgba16float and fp32 image equal the full-frame JS render's; the fp32 image is zero
    outside the band (what commGatherBands sums)."""
    vol = cf.fbm_volume(64, 9, nthreads=8)
    R, y0, y1 = 64, 16, 48
    (tmp_path / "full").mkdir()
    (tmp_path / "band").mkdir()
    ph_f, rgba_f, _, _ = run_case(tmp_path / "full", vol, cf.tf_spectral(), R=R, passes=3)
    rgb_f = run_case.rgb32
    ph_b, rgba_b, _, _ = run_case(tmp_path / "band", vol, cf.tf_spectral(), R=R, passes=3,
                                  band=[y0, y1])
    rgb_b = run_case.rgb32
    assert np.array_equal(rgba_b[y0:y1], rgba_f[y0:y1])
    assert np.array_equal(rgb_b[y0:y1].view(np.uint32), rgb_f[y0:y1].view(np.uint32))
    assert not rgb_b[:y0].any() and not rgb_b[y1:].any()
    rows = ph_f.reshape(R, R, 36)[y0:y1]
    assert np.array_equal(ph_b.reshape(R, R, 36)[y0:y1], rows)


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_napi_guards_and_extensions():
    """N-API output arrays are checked against the handle's own R (a caller's
    smaller R is refused, not written past); renderPasses(n) / lastLaunch() on
    both JS renderer classes (40 passes = 32 + 8, 33 = 32 + 1)."""
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "gpu_guards.js")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("small_rgb", "small_rgba", "small_photons"):
        assert out[k] and "does not match" in out[k], (k, out[k])
    assert out["short_array"] and "too short" in out["short_array"], out["short_array"]
    assert out["ok_rgb"] is None
    assert out["spectral_launches"] == 2 and out["spectral_last"]["passes"] == 8, out
    assert out["rgb_launches"] == 2 and out["rgb_last"]["passes"] == 1, out


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_js_device_list_renderer_composites(tmp_path):
    """The JS drop-in driving a device list (createDevice([0, 0]): two replicas;
    on an N-GPU node the list names N GPUs): render() per pass as the reference
    loop calls it, getTexture() returns the composite sum(rgb*n)/sum(n) of the
    replicas, bit-exact against two oracle replays (replica 1 on rank 1's seed
    stream) composited in replica order; readPhotons() is replica 0's."""
    from test_gpu_group import _composite
    vol, tf = cf.sphere_in_cube(64), cf.tf_spectral()
    ph, rgba, seeds, used = run_case(tmp_path, vol, tf, passes=5, devices=[0, 0])
    assert run_case.meta["devices"] == [0, 0]
    R = 64
    bits = [int(np.float32(s).view(np.uint32)) for s in seeds]
    reps = []
    mvp = cf.default_mvp_inverse()
    for k in (0, 1):  # the JS call sequence of oracle_replay, on replica k's seed bits
        rs = [b if k == 0 else cf.pcg(b ^ ((k * 0x9E3779B9) & 0xFFFFFFFF)) for b in bits]
        o = orc.Oracle(R)
        o.volume, o.tf, o.light = vol, tf, np.full(256, 100, np.uint8)
        o.params.update(extinction=32.0, bounces=8, steps=8)
        o.reset(mvp, rs[0])
        o.set_spectrum(cf.spectrum_buffer("12"))
        for p in range(5):
            rgb32, _ = o.render(mvp, rs[1 + p])
        reps.append((o, rgb32))
    assert same(ph[:, :34], reps[0][0].photons[:, :34])
    want_rgb, want_rgba, _ = _composite(reps)
    assert np.array_equal(rgba, want_rgba)
    assert same(run_case.rgb32.view(np.uint32), want_rgb.view(np.uint32))


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
def test_napi_comm_init():
    """The communicator through the N-API shim: a one-rank
    communicator composites a pass (the composite of one replica is its own
    image); a two-rank communicator whose rank 1 never arrives makes commInit
    throw the communicator error within VPTMCM_COMM_TIMEOUT_MS instead of
    blocking the JS host forever, and the process then ends."""
    import os
    import time
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "comm_init.js"), "one"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["uid_bytes"] == 128 and out["max_rel"] <= 2.5e-7, out
    env = dict(os.environ, VPTMCM_COMM_TIMEOUT_MS="3000")
    t0 = time.monotonic()
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "comm_init.js"), "never"], capture_output=True,
                       text=True, timeout=120, env=env)
    took = time.monotonic() - t0
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out.get("code") == -5 and "did not return within 3000 ms" in out["message"], out
    assert 3000 <= out["took_ms"] < 20000, out
    assert r.returncode == 3 and took < 100, (r.returncode, took, r.stderr[-2000:])
