"""Randomised GPU parity: seeded random configurations of every input the march
reads — resolution (incl. R not a multiple of 8), ragged volume shapes, all
four layouts, random / few-row / many-row TFs with constant or varying
anisotropy, random bin layouts (uneven, duplicate and unsorted boundaries,
random CMF coefficients), random light SPD and direction (incl. isotropic),
extinction over three decades plus 0 and 1e4, bounces, steps, depth of field and random camera
matrices (incl. a camera inside the volume) — against the oracle, bit for bit,
through unfused and fused (queued) passes. Each case prints its draw, so a
failure names the configuration that exposed it.
"""
import os

import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf
from test_gpu_parity import assert_photons_equal, assert_rgb32_equal, assert_rgba_equal

pytestmark = pytest.mark.gpu

# VPTMCM_FUZZ_CASES / VPTMCM_FUZZ_BASE: a longer campaign over fresh draws
# (tools/fuzz_campaign.sh; the suite's defaults are 96 cases from base 0)
N_CASES = int(os.environ.get("VPTMCM_FUZZ_CASES", "96"))
BASE = int(os.environ.get("VPTMCM_FUZZ_BASE", "0"))
# (MODE, layout template) pairs the random cases' fused launches ran
# (vptmcm_debug_last_launch); test_mode_template_coverage forces the rest
HIT = set()


def _perspective_inverse(rng, inside=False):
    """invert(P * V * M) of a random look-at camera (float64, rounded to f32 once)."""
    f = 1.0 / np.tan(rng.uniform(0.4, 1.2) / 2)
    near, far = 0.1, 100.0
    P = np.array([[f, 0, 0, 0], [0, f, 0, 0],
                  [0, 0, (far + near) / (near - far), 2 * far * near / (near - far)],
                  [0, 0, -1, 0]])
    target = rng.uniform(0.3, 0.7, 3) if not inside else rng.uniform(0.45, 0.55, 3)
    if inside:
        eye = rng.uniform(0.3, 0.7, 3)
    else:
        d = rng.normal(size=3)
        eye = 0.5 + d / np.linalg.norm(d) * rng.uniform(1.2, 3.0)
    fwd = target - eye
    fwd /= np.linalg.norm(fwd)
    up = np.array([0.0, 1.0, 0.0]) if abs(fwd[1]) < 0.95 else np.array([1.0, 0.0, 0.0])
    s = np.cross(fwd, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, fwd)
    V = np.eye(4)
    V[0, :3], V[1, :3], V[2, :3] = s, u, -fwd
    V[:3, 3] = -V[:3, :3] @ eye
    # column-major f32[16], as the renderer uploads gl-matrix matrices
    return np.linalg.inv(P @ V).T.reshape(16).astype(np.float32)


def _spectrum(rng):
    kind = rng.integers(0, 5)
    if kind == 0:
        return "12 equal", cf.spectrum_buffer("12")
    nb = int(rng.integers(1, 13))
    bins = np.sort(rng.integers(400, 701, nb + 1)).astype(np.float64)
    what = f"{nb} random bins"
    if kind == 1:  # duplicate boundaries: zero-width bins (UI markers may coincide)
        bins[rng.integers(0, nb + 1)] = bins[rng.integers(0, nb + 1)]
        bins = np.sort(bins)
        what += " (duplicates)"
    if kind == 2:  # unsorted markers (the generic bin search)
        rng.shuffle(bins)
        what += " (unsorted)"
    buf = np.zeros(64, np.float32)
    coeff = rng.uniform(0.0, 2.0, 3 * nb)
    buf[: 1 + (nb + 1) + 3 * nb] = np.concatenate([[nb], bins, coeff])
    return what, buf


def _tf(rng):
    kind = rng.integers(0, 5)
    if kind == 0:
        return "spectral", cf.tf_spectral()
    if kind == 1:
        return "materials varying b", cf.tf_materials(True)
    if kind == 2:
        return "materials constant b", cf.tf_materials(False)
    if kind == 3:  # few distinct rows painted over random ranges (deduplicated TF)
        t = np.zeros((256, 256, 4), np.uint8)
        edges = np.sort(rng.integers(0, 256, 6))
        for a, b in zip(edges[:-1], edges[1:]):
            mat = rng.integers(0, 256, (256, 3), dtype=np.uint8)
            if rng.random() < 0.5:
                mat[:, 2] = mat[0, 2]
            t[a:b, :, :3] = mat[None]
        return "random few-row", t
    t = rng.integers(0, 256, (256, 256, 4), dtype=np.uint8)  # every row distinct
    return "random noise", t


def _draw(k):
    rng = np.random.default_rng(1000 + BASE + k)
    R = int(rng.choice([8, 16, 24, 40, 48, 64, 72, 96, 128, 200, 256])) + (int(rng.integers(1, 8)) if rng.random() < 0.3 else 0)
    shape = tuple(int(x) for x in rng.integers(1, 72, 3)) if rng.random() < 0.4 else (48, 48, 48)
    layout = int(rng.choice([vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_LINEAR, vptmcm.LAYOUT_BRICK8,
                             vptmcm.LAYOUT_COLUMN4]))
    spec_what, spec = _spectrum(rng)
    tf_what, tf = _tf(rng)
    iso = rng.random() < 0.2
    ld = np.zeros(3, np.float32) if iso else rng.normal(size=3).astype(np.float32)
    spd = (np.full(256, 100, np.uint8) if rng.random() < 0.5
           else rng.integers(0, 256, 256, dtype=np.uint8))
    ext = float(np.float32(10 ** rng.uniform(-0.3, 2.5)))
    ext = {0: 0.0, 1: 1e4}.get(int(rng.integers(0, 20)), ext)  # inf/NaN distances; huge majorant
    params = dict(extinction=ext, bounces=int(rng.integers(0, 11)), steps=int(rng.integers(0, 41)),
                  blur=float(np.float32(rng.uniform(0, 0.5))) if rng.random() < 0.25 else 0.0)
    mvp = (cf.default_mvp_inverse() if rng.random() < 0.25
           else _perspective_inverse(rng, inside=rng.random() < 0.2))
    vol_seed = int(rng.integers(0, 1 << 16))
    what = (f"case {k}: R={R} vol={shape} layout={layout} bins={spec_what} tf={tf_what} "
            f"light={'isotropic' if iso else 'directional'} {params}")
    return R, shape, layout, spec, tf, ld, spd, params, mvp, vol_seed, what


def _volume(shape, seed):
    if shape == (48, 48, 48):
        return cf.fbm_volume(48, seed % 97, nthreads=8)
    rng = np.random.default_rng(seed)
    D, H, W = shape[2], shape[1], shape[0]
    base = rng.integers(0, 256, (D, H, W)).astype(np.float64)
    # a smooth blob plus noise: both empty and dense regions
    z, y, x = np.meshgrid(*(np.linspace(-1, 1, n) for n in (D, H, W)), indexing="ij")
    blob = np.clip(1.2 - np.sqrt(x * x + y * y + z * z), 0, 1) * 255
    return np.clip(0.6 * blob + 0.4 * base * (blob > 0), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("k", range(N_CASES))
def test_random_configuration_bitexact(k, monkeypatch):
    R, shape, layout, spec, tf, ld, spd, params, mvp, vol_seed, what = _draw(k)
    # the macro-cell null-collision skip pinned on for even cases (odd: the
    # tuner's pick, which probes both sides on a handle's first launches)
    if k % 2 == 0:
        monkeypatch.setenv("VPTMCM_MAJ", "on")
        what += " maj=on"
    print(what)
    vol = _volume(shape, vol_seed)
    with vptmcm.Renderer(R, device=0, layout=layout) as gpu:
        cpu = orc.Oracle(R)
        gpu.set_spectrum(spec)
        cpu.set_spectrum(spec)
        gpu.set_volume(vol)
        gpu.set_material_tf(tf)
        gpu.set_light(spd, ld)
        gpu.set_params(**params)
        cpu.volume, cpu.tf, cpu.light, cpu.light_dir = vol, tf, spd, ld
        cpu.params.update(**params)
        seeds = cf.seed_stream(6, start=10 * (BASE + k))
        gpu.reset(mvp, seeds[0])
        cpu.reset(mvp, seeds[0], nthreads=16)
        assert_photons_equal(gpu.read_photons(), cpu.photons, what + " reset")
        for p in (1, 2):  # one launch per pass (read back between them)
            gpu.render(mvp, seeds[p])
            rgb, want = cpu.render(mvp, seeds[p], nthreads=16)
            assert_photons_equal(gpu.read_photons(), cpu.photons, f"{what} pass {p}")
            assert_rgba_equal(gpu.read_rgba16f(), want, f"{what} pass {p}")
            assert_rgb32_equal(gpu.read_rgb(), rgb, f"{what} pass {p}")
        for p in (3, 4, 5):  # queued: one fused launch of three passes
            gpu.render(mvp, seeds[p])
            rgb, want = cpu.render(mvp, seeds[p], nthreads=16)
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"{what} fused")
        assert_rgba_equal(gpu.read_rgba16f(), want, f"{what} fused")
        assert_rgb32_equal(gpu.read_rgb(), rgb, f"{what} fused")
        info = gpu.last_launch()
        assert info["passes"] == 3 and info["spec"], info
        HIT.add((info["mode"], info["tpl"]))


def _same_words(a, b):
    fa, fb = a.view(np.float32), b.view(np.float32)
    return (a == b) | (np.isnan(fa) & np.isnan(fb))


@pytest.mark.parametrize("k", range(N_CASES // 2))
def test_random_configuration_rgb_bitexact(k):
    """The RGB sibling ('mcm-compute') under the same random draws, with a random
    rgba8 TF image (random width/height; the kernel samples row 0), a random
    environment colour and a random anisotropy."""
    R, shape, layout, _, _, _, _, params, mvp, vol_seed, what = _draw(k)
    rng = np.random.default_rng(5000 + BASE + k)
    tf = rng.integers(0, 256, (int(rng.integers(1, 4)), int(rng.integers(2, 300)), 4), dtype=np.uint8)
    env = tuple(int(x) for x in rng.integers(0, 256, 4))
    aniso = float(np.float32(rng.uniform(-0.95, 0.95)))
    params = dict(extinction=params["extinction"], anisotropy=aniso, bounces=params["bounces"],
                  steps=params["steps"])
    what = f"rgb {what} tf={tf.shape} env={env} anisotropy={aniso}"
    print(what)
    vol = _volume(shape, vol_seed)
    with vptmcm.Renderer(R, device=0, layout=layout, renderer=vptmcm.RENDERER_RGB) as gpu:
        cpu = orc.OracleRGB(R)
        gpu.set_transfer_function(tf)
        gpu.set_environment(env)
        gpu.set_volume(vol)
        gpu.set_params(**params)
        cpu.volume, cpu.tf, cpu.env = vol, tf, np.array(env, np.uint8)
        cpu.params.update(**params)
        seeds = cf.seed_stream(6, start=10 * (BASE + k) + 3)
        gpu.reset(mvp, seeds[0])
        cpu.reset(mvp, seeds[0])
        assert _same_words(gpu.read_photons(), cpu.photons).all(), what + " reset"
        for p in (1, 2):
            gpu.render(mvp, seeds[p])
            _, want = cpu.render(mvp, seeds[p])
            ok = _same_words(gpu.read_photons(), cpu.photons)
            assert ok.all(), f"{what} pass {p}: {int((~ok).sum())} photon words differ"
            assert np.array_equal(gpu.read_rgba16f(), want), f"{what} pass {p}: image differs"
        gpu.render_passes(mvp, seeds[3:])  # one fused launch
        for s in seeds[3:]:
            _, want = cpu.render(mvp, s)
        assert _same_words(gpu.read_photons(), cpu.photons).all(), what + " fused"
        assert np.array_equal(gpu.read_rgba16f(), want), what + " fused image"


def _setup_spectral(gpu, cpu, draw):
    R, shape, layout, spec, tf, ld, spd, params, mvp, vol_seed, what = draw
    vol = _volume(shape, vol_seed)
    for r in (gpu, cpu):
        r.set_spectrum(spec)
    gpu.set_volume(vol)
    gpu.set_material_tf(tf)
    gpu.set_light(spd, ld)
    gpu.set_params(**params)
    cpu.volume, cpu.tf, cpu.light, cpu.light_dir = vol, tf, spd, ld
    cpu.params.update(**params)


@pytest.mark.parametrize("k", range(N_CASES // 4))
def test_random_bands_bitexact(k):
    """Mode B under random draws: the frame cut into 1-4 random row bands (whole
    8-row tiles; the last band ends at R, which need not be a multiple of 8), one
    handle per band; every band's rows equal the oracle's full frame and the band
    images sum to the oracle's fp32 image, bit for bit."""
    draw = _draw(200 + k)  # (BASE applies inside _draw)
    R, mvp, what = draw[0], draw[8], draw[10]
    rng = np.random.default_rng(7000 + BASE + k)
    tiles = (R + 7) // 8
    cuts = sorted(set(int(c) * 8 for c in rng.integers(1, tiles, int(rng.integers(0, 4))))) if tiles > 1 else []
    edges = [0] + cuts + [R]
    bands = list(zip(edges[:-1], edges[1:]))
    print(what, "bands", bands)
    cpu = orc.Oracle(R)
    gpus = [vptmcm.Renderer(R, device=0, layout=draw[2]) for _ in bands]
    try:
        _setup_spectral(gpus[0], cpu, draw)
        for g, (y0, y1) in zip(gpus[1:], bands[1:]):
            _setup_spectral(g, orc.Oracle(R), draw)
        for g, (y0, y1) in zip(gpus, bands):
            g.set_band(y0, y1)
        seeds = cf.seed_stream(5, start=10 * (BASE + k) + 7)
        cpu.reset(mvp, seeds[0], nthreads=16)
        for s in seeds[1:]:
            rgb, want = cpu.render(mvp, s, nthreads=16)
        acc = np.zeros((R, R, 3), np.float32)
        for g, (y0, y1) in zip(gpus, bands):
            g.reset(mvp, seeds[0])
            g.render(mvp, seeds[1])
            g.read_rgb()  # a read between passes: an unfused launch, then a fused one
            g.render_passes(mvp, seeds[2:])
            ph = g.read_photons().reshape(R, R, -1)[y0:y1].reshape(-1, 36)
            assert_photons_equal(ph, cpu.photons.reshape(R, R, -1)[y0:y1].reshape(-1, 36),
                                 f"{what} band {y0}:{y1}")
            assert_rgba_equal(g.read_rgba16f()[y0:y1], want[y0:y1], f"{what} band {y0}:{y1}")
            img = g.read_rgb()
            assert not img[:y0].any() and not img[y1:].any()
            acc += img
        assert_rgb32_equal(acc, rgb, f"{what} band sum")
    finally:
        for g in gpus:
            g.close()


@pytest.mark.parametrize("k", range(max(1, N_CASES // 8)))
def test_random_group_composite_bitexact(k):
    """Device-list handles under random draws: 2-8 replicas on device 0 (every
    forwarded call on the replicas' worker threads), replica j on rank j's seed
    stream; replica 0's photons, the composite's fp32 and rgba16float images and
    its sample counts bit for bit against the oracle replicas composited in
    replica order (tests/test_gpu_group.py's numpy restatement of k_composite)."""
    from test_gpu_group import _composite
    R, shape, layout, spec, tf, ld, spd, params, mvp, vol_seed, what = _draw(400 + k)
    rng = np.random.default_rng(9000 + BASE + k)
    n_rep = int(rng.integers(2, 9))
    what = f"group x{n_rep} {what}"
    print(what)
    vol = _volume(shape, vol_seed)
    start = 10 * (BASE + k) + 9
    seeds = cf.seed_stream(5, start=start)
    with vptmcm.Renderer(R, devices=[0] * n_rep, layout=layout) as g:
        g.set_spectrum(spec)
        g.set_volume(vol)
        g.set_material_tf(tf)
        g.set_light(spd, ld)
        g.set_params(**params)
        g.reset(mvp, seeds[0])
        g.render(mvp, seeds[1])
        g.read_rgb()  # a composite between passes: an unfused launch, then a fused one
        g.render_passes(mvp, seeds[2:])
        reps = []
        for j in range(n_rep):
            o = orc.Oracle(R)
            o.set_spectrum(spec)
            o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
            o.params.update(**params)
            rs = cf.seed_stream(5, start=start, rank=j)
            o.reset(mvp, rs[0], nthreads=16)
            for s_ in rs[1:]:
                rgb, _ = o.render(mvp, s_, nthreads=16)
            reps.append((o, rgb))
        assert_photons_equal(g.read_photons(), reps[0][0].photons, what + " replica 0")
        want_rgb, want_rgba, want_n = _composite(reps)
        q, crgb, n = g.read_composite_all()
        assert np.array_equal(n, want_n), what + " counts"
        assert_rgb32_equal(crgb, want_rgb, what + " composite fp32")
        assert_rgba_equal(q, want_rgba, what + " composite rgba16f")


def _close_bins():
    """3 bins whose inner boundaries (500.1, 500.15 nm) put two distinct
    thresholds in one cell of the wavelength-bin table: the table is refused and
    the comparison search runs (MODE 4 / 5 instead of 6 / 7)."""
    buf = np.zeros(64, np.float32)
    buf[:1 + 4 + 9] = [3, 450.0, 500.1, 500.15, 650.0, 0.3, 1.1, 0.7, 0.2, 0.9, 1.4, 1.6, 0.1, 0.4]
    return buf


# the inputs that make launch_march select each MODE (see its dispatcher and
# DESIGN.md section 5): TF, bin layout, light direction
_MODE_INPUTS = {
    2: ("spectral", "12", False),
    3: ("materials", "12", False),
    6: ("materials", "8_uneven", False),
    4: ("materials", "close", False),
    7: ("noise", "8_uneven", False),
    5: ("noise", "close", False),
    1: ("spectral", "12", True),
    0: ("spectral", "8_uneven", True),
}
# layout template -> (layout, force 64-bit offsets: VPTMCM_MARCH_VARIANT=8)
_TEMPLATES = {0: (vptmcm.LAYOUT_LINEAR, False), 1: (vptmcm.LAYOUT_CORNER8, False),
              2: (vptmcm.LAYOUT_CORNER8, True), 3: (vptmcm.LAYOUT_BRICK8, False),
              4: (vptmcm.LAYOUT_BRICK8, True), 5: (vptmcm.LAYOUT_COLUMN4, False),
              6: (vptmcm.LAYOUT_COLUMN4, True)}


def test_mode_template_coverage(monkeypatch):
    """Every (MODE, layout template) pair the dispatcher can select has run bit
    for bit against the oracle: the pairs the random cases did not reach are
    forced here (and asserted to be the pair that launched)."""
    rng = np.random.default_rng(77)
    noise = rng.integers(0, 256, (256, 256, 4), dtype=np.uint8)
    tfs = {"spectral": cf.tf_spectral(), "materials": cf.tf_materials(True), "noise": noise}
    specs = {"12": cf.spectrum_buffer("12"), "8_uneven": cf.spectrum_buffer("8_uneven"),
             "close": _close_bins()}
    vol = cf.sphere_in_cube(24)
    mvp = cf.default_mvp_inverse()
    spd, ldir = cf.light_default()
    R = 32
    forced = []
    for mode, (tfk, bk, iso) in _MODE_INPUTS.items():
        for tpl, (layout, wide) in _TEMPLATES.items():
            if (mode, tpl) in HIT:
                continue
            forced.append((mode, tpl))
            what = f"MODE {mode} template {tpl}: tf={tfk} bins={bk} isotropic={iso}"
            ld = np.zeros(3, np.float32) if iso else ldir
            if wide:
                monkeypatch.setenv("VPTMCM_MARCH_VARIANT", "8")
            else:
                monkeypatch.delenv("VPTMCM_MARCH_VARIANT", raising=False)
            with vptmcm.Renderer(R, device=0, layout=layout) as gpu:
                cpu = orc.Oracle(R)
                for r in (gpu, cpu):
                    r.set_spectrum(specs[bk])
                gpu.set_volume(vol)
                gpu.set_material_tf(tfs[tfk])
                gpu.set_light(spd, ld)
                gpu.set_params(extinction=24.0, bounces=8, steps=8)
                cpu.volume, cpu.tf, cpu.light, cpu.light_dir = vol, tfs[tfk], spd, ld
                cpu.params.update(extinction=24.0, bounces=8, steps=8)
                seeds = cf.seed_stream(5, start=mode * 10 + tpl)
                gpu.reset(mvp, seeds[0])
                cpu.reset(mvp, seeds[0], nthreads=8)
                gpu.render(mvp, seeds[1])
                cpu.render(mvp, seeds[1], nthreads=8)
                assert_photons_equal(gpu.read_photons(), cpu.photons, what + " pass 1")
                gpu.render_passes(mvp, seeds[2:])
                for sd in seeds[2:]:
                    rgb, want = cpu.render(mvp, sd, nthreads=8)
                info = gpu.last_launch()
                assert (info["mode"], info["tpl"], info["passes"]) == (mode, tpl, 3), (what, info)
                assert_photons_equal(gpu.read_photons(), cpu.photons, what + " fused")
                assert_rgba_equal(gpu.read_rgba16f(), want, what + " fused")
                assert_rgb32_equal(gpu.read_rgb(), rgb, what + " fused")
            HIT.add((mode, tpl))
    print(f"forced {len(forced)} of {8 * len(_TEMPLATES)} pairs: {forced}")
    assert len(HIT) == 8 * len(_TEMPLATES)
