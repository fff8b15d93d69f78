"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar: bit-exact photon state (NaN == NaN) and bit-exact rgba16float image on the
same seeded inputs — the arithmetic specification makes the two identical, so
the fixed-seed tolerance of north_star (<= 1e-4 relative L2) is met with 0.
Full-size (R = 512, 512^3 volume) frames are small enough for the threaded
oracle, so the benchmark configuration itself is checked bit for bit.
"""
import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf

pytestmark = pytest.mark.gpu

LAYOUTS = [vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_LINEAR, vptmcm.LAYOUT_BRICK8, vptmcm.LAYOUT_COLUMN4]


def same_words(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    fa, fb = a.view(np.float32), b.view(np.float32)
    return (a == b) | (np.isnan(fa) & np.isnan(fb))


def assert_photons_equal(got, want, what=""):
    ok = same_words(got[:, :34], want[:, :34])
    if not ok.all():
        bad = np.argwhere(~ok)
        pix, word = bad[0]
        raise AssertionError(f"{what}: {len(bad)} words differ; first photon {pix} word {word}: "
                             f"gpu {got[pix, word]:#x} oracle {want[pix, word]:#x}")


def assert_rgba_equal(got, want, what=""):
    g, w = got.view(np.float16), want.view(np.float16)
    ok = (got == want) | (np.isnan(g) & np.isnan(w))
    assert ok.all(), f"{what}: {int((~ok).sum())} rgba16f halfs differ"


def make_pair(R, vol, tf, spec="12", ext=32.0, layout=vptmcm.LAYOUT_CORNER8, light_dir=(1, 0, 0),
              spd=None, bounces=8, steps=8, blur=0.0, upload_spectrum=True):
    gpu = vptmcm.Renderer(R, device=0, layout=layout)
    cpu = orc.Oracle(R)
    spd = np.full(256, 100, np.uint8) if spd is None else spd
    ld = np.asarray(light_dir, np.float32)
    if upload_spectrum:
        buf = cf.spectrum_buffer(spec)
        gpu.set_spectrum(buf)
        cpu.set_spectrum(buf)
    gpu.set_volume(vol)
    gpu.set_material_tf(tf)
    gpu.set_light(spd, ld)
    gpu.set_params(extinction=ext, bounces=bounces, steps=steps, blur=blur)
    cpu.volume, cpu.tf, cpu.light, cpu.light_dir = vol, tf, spd, ld
    cpu.params.update(extinction=ext, bounces=bounces, steps=steps, blur=blur)
    return gpu, cpu


def assert_rgb32_equal(got, want, what=""):
    """a13 before the f16 store: the fp32 radiance_to_rgb result, bit for bit."""
    ok = same_words(got.view(np.uint32), want.view(np.uint32))
    assert ok.all(), f"{what}: {int((~ok).sum())} fp32 rgb words differ"


def run_and_compare(gpu, cpu, mvp, seeds, what, nthreads=16):
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=nthreads)
    assert_photons_equal(gpu.read_photons(), cpu.photons, what + " reset")
    for k, s in enumerate(seeds[1:], 1):
        gpu.render(mvp, s)
        rgb, want = cpu.render(mvp, s, nthreads=nthreads)
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"{what} pass {k}")
        assert_rgba_equal(gpu.read_rgba16f(), want, f"{what} pass {k}")
        assert_rgb32_equal(gpu.read_rgb(), rgb, f"{what} pass {k}")


def test_math_primitives_bitexact():
    with vptmcm.Renderer(8, device=0) as gpu:
        o = orc.Oracle(1)
        rng = np.random.default_rng(7)
        u = (rng.integers(0, 2 ** 32, 1 << 20, dtype=np.uint64).astype(np.float32) *
             np.float32(2.0 ** -32)).astype(np.float32)
        edge = np.float32([0.0, -0.0, 1.0, 1e-45, 1e-38, 3.0, np.inf, -1.0, np.nan])
        xs = np.concatenate([u, edge]).view(np.uint32)
        ang = (np.linspace(0, 6.2831855, 1 << 20, dtype=np.float32)).view(np.uint32)
        for fn, inp in [(0, xs), (1, ang), (2, ang), (3, rng.integers(0, 2 ** 32, 1 << 20, dtype=np.uint64).astype(np.uint32)),
                        (4, (rng.standard_normal(1 << 20).astype(np.float32) * 300).view(np.uint32))]:
            g, c = gpu.debug_eval(fn, inp), o.eval_batch(fn, inp)
            if fn == 4:
                g, c = g.astype(np.uint16), c.astype(np.uint16)
                ok = (g == c) | (np.isnan(g.view(np.float16)) & np.isnan(c.view(np.float16)))
            elif fn == 3:
                ok = g == c
            else:
                ok = same_words(g, c)
            assert ok.all(), f"fn {fn}: {int((~ok).sum())} mismatches"


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("tfname,ext", [("spectral", 1.0), ("spectral", 32.0), ("zero", 1.0),
                                        ("grey", 32.0)])
def test_c1_sphere_in_cube(layout, tfname, ext):
    tf = {"spectral": cf.tf_spectral, "zero": cf.tf_zero, "grey": cf.tf_grey}[tfname]()
    gpu, cpu = make_pair(64, cf.sphere_in_cube(64), tf, ext=ext, layout=layout)
    run_and_compare(gpu, cpu, cf.default_mvp_inverse(), cf.seed_stream(9, start=0),
                    f"C1 {tfname} ext={ext} layout={layout}")
    gpu.close()


@pytest.mark.parametrize("variant", ["0", "1"])
@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("tfname", ["spectral", "materials", "materials_const_b"])
def test_march_variants_bitexact(variant, layout, tfname, monkeypatch):
    """Every step-loop variant (speculative / plain) is bit-exact, with a
    row-invariant anisotropy channel (LDS row table) and a wavelength-varying one
    (4-corner gather)."""
    monkeypatch.setenv("VPTMCM_MARCH_VARIANT", variant)
    tf = {"spectral": cf.tf_spectral(), "materials": cf.tf_materials(True),
          "materials_const_b": cf.tf_materials(False)}[tfname]
    gpu, cpu = make_pair(64, cf.fbm_volume(64, 3, nthreads=8), tf, ext=24.0, layout=layout)
    run_and_compare(gpu, cpu, cf.golden_mvp("orbit"), cf.seed_stream(5, start=0),
                    f"variant {variant} layout {layout} tf {tfname}")
    gpu.close()


def _tf_many_rows_varying_b():
    """> kTfRowsMax distinct rows AND a wavelength-varying anisotropy channel:
    neither the LDS row table nor the deduplicated TF applies (tf_b4 gather)."""
    t = cf.tf_spectral()
    t[..., 2] = (40 + (np.arange(256) * 0.6)).astype(np.uint8)[None, :]
    return t


@pytest.mark.parametrize("variant", ["0", "16", "32", "64"])
@pytest.mark.parametrize("spec", ["12", "8_uneven", "3", "12_wide"])
@pytest.mark.parametrize("tfname", ["materials", "materials_const_b", "many_rows_b"])
def test_tf_modes_bitexact(variant, spec, tfname, monkeypatch):
    """The march specialisations chosen per launch — MODE 2 (FAST: row-invariant
    anisotropy), 3 (row-deduplicated LDS TF, 12 equal bins), 4 (deduplicated TF,
    any bins), 5 (more distinct rows than the deduplicated TF holds, any bins),
    6/7 (4/5 with the wavelength-bin table; variant bit 6 keeps 4/5), 1/0
    (generic; variant bits 4/5 force them) — against the oracle,
    bit for bit, over TFs with few distinct rows (the UI's materials, with
    constant and wavelength-varying anisotropy) and many rows with varying
    anisotropy (tf_b4 gather), for equal, uneven, few and wide bin layouts."""
    monkeypatch.setenv("VPTMCM_MARCH_VARIANT", variant)
    tf = {"materials": cf.tf_materials(True), "materials_const_b": cf.tf_materials(False),
          "many_rows_b": _tf_many_rows_varying_b()}[tfname]
    gpu, cpu = make_pair(64, cf.fbm_volume(64, 7, nthreads=8), tf, spec=spec, ext=24.0)
    run_and_compare(gpu, cpu, cf.default_mvp_inverse(), cf.seed_stream(4, start=0),
                    f"variant {variant} bins {spec} tf {tfname}")
    # the specialisation that ran: "12" is the only layout with the arithmetic
    # (equal-width) bin search; every other one takes the exact bin table
    # (MODE 6 / 7) unless variant bit 6 keeps the comparison search (4 / 5)
    uniform = spec == "12"
    if variant == "16":
        want = 1 if spec in ("12", "12_wide") else 0
    elif variant == "32":
        want = 0
    elif tfname == "many_rows_b":
        want = 5 if variant == "64" else 7
    elif uniform:
        want = 2 if tfname == "materials_const_b" else 3
    else:
        want = 4 if variant == "64" else 6
    info = gpu.last_launch()
    assert info["mode"] == want, (variant, spec, tfname, info)
    gpu.close()


def test_bin_table_falls_back_for_close_boundaries():
    """build_bin_lut (vptmcm.cpp) keeps the comparison search when two distinct
    bin thresholds fall into one of its 1024 wavelength cells (~0.29 nm wide on
    [400, 700]): boundaries 0.05 nm apart must run MODE 4 (no table), not 6, and
    still match the oracle bit for bit; the same layout with the pair spread
    apart takes the table (MODE 6)."""
    base = cf.spectrum_buffer("8_uneven").copy()
    nb = int(base[0] + 0.5)
    assert nb == 8
    for lams, want in [([400, 450, 500, 500.05, 550, 600, 640, 680, 700], 4),
                       ([400, 450, 500, 510, 550, 600, 640, 680, 700], 6)]:
        buf = base.copy()
        buf[1:2 + nb] = np.float32(lams)
        cells = ((np.float32(lams) - 400) / 300 * 1024).astype(int)
        assert (cells[2] == cells[3]) == (want == 4)  # the close pair shares a cell
        gpu, cpu = make_pair(64, cf.fbm_volume(64, 7, nthreads=8), cf.tf_materials(True), ext=24.0,
                             upload_spectrum=False)
        gpu.set_spectrum(buf)
        cpu.set_spectrum(buf)
        run_and_compare(gpu, cpu, cf.default_mvp_inverse(), cf.seed_stream(3, start=0),
                        f"bins {lams}")
        info = gpu.last_launch()
        assert info["mode"] == want, (lams, info)
        gpu.close()


@pytest.mark.parametrize("camera", ["near", "orbit", "orbit_tilted"])
def test_cameras_and_bins(camera):
    for spec in ("6", "3", "8_uneven", "12_wide"):
        gpu, cpu = make_pair(48, cf.two_spheres(48), cf.tf_spectral(), spec=spec, ext=16.0)
        run_and_compare(gpu, cpu, cf.golden_mvp(camera), cf.seed_stream(3, start=0),
                        f"{camera} bins={spec}")
        gpu.close()


def test_edge_cases():
    vol = cf.fbm_volume(40, 7, nthreads=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(4, start=0)
    cases = [
        dict(R=37, what="R not multiple of 8"),
        dict(R=32, ext=0.0, what="extinction 0 (inf/NaN distances)"),
        dict(R=32, bounces=0, what="no scattering"),
        dict(R=32, light_dir=(0, 0, 0), what="isotropic light"),
        dict(R=32, blur=0.3, steps=33, what="depth of field + odd steps"),
        dict(R=32, steps=0, what="zero steps"),
        dict(R=24, ext=1e4, what="huge majorant"),
    ]
    for c in cases:
        what = c.pop("what")
        R = c.pop("R")
        gpu, cpu = make_pair(R, vol, cf.tf_spectral(), **c)
        run_and_compare(gpu, cpu, mvp, seeds, what)
        gpu.close()


@pytest.mark.parametrize("tfname", ["spectral", "materials"])
def test_first_reset_quirk_and_spectrum_change(tfname):
    """reset() before the first spectrum upload, a C-ABI render with
    no bins at all (nb = 0: every specialisation, incl. the deduplicated-TF
    MODE 4, leaves the bins untouched), then renders with 12 and 6 bins."""
    tf = cf.tf_spectral() if tfname == "spectral" else cf.tf_materials(True)
    gpu, cpu = make_pair(32, cf.sphere_in_cube(32), tf, upload_spectrum=False)
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, cf.seed_bits(0))
    cpu.reset(mvp, cf.seed_bits(0))
    assert_photons_equal(gpu.read_photons(), cpu.photons, "zero-spectrum reset")
    gpu.render(mvp, cf.seed_bits(9))
    _, want = cpu.render(mvp, cf.seed_bits(9))
    assert_photons_equal(gpu.read_photons(), cpu.photons, "zero-spectrum render")
    assert_rgba_equal(gpu.read_rgba16f(), want, "zero-spectrum render")
    for k, spec in [(1, "12"), (2, "12"), (3, "6"), (4, "6")]:
        buf = cf.spectrum_buffer(spec)
        gpu.set_spectrum(buf)
        cpu.set_spectrum(buf)
        gpu.render(mvp, cf.seed_bits(k))
        _, want = cpu.render(mvp, cf.seed_bits(k))
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"pass {k} spectrum {spec}")
        assert_rgba_equal(gpu.read_rgba16f(), want, f"pass {k}")
    gpu.close()


def test_photon_roundtrip_and_resume():
    gpu, cpu = make_pair(32, cf.sphere_in_cube(32), cf.tf_spectral())
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 1)
    gpu.render(mvp, 2)
    words = gpu.read_photons()
    cpu.photons = words.copy()
    gpu.write_photons(words)
    assert np.array_equal(gpu.read_photons()[:, :34], words[:, :34])
    gpu.render(mvp, 3)
    cpu.render(mvp, 3)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "resume")
    gpu.close()


@pytest.mark.parametrize("layout", LAYOUTS)
def test_streamed_volume_renders_while_blocks_arrive(layout):
    """Streaming ingest (SURVEY 8f f1, C5's brick streaming): every placement's
    cells / bricks are re-laid out as it arrives, and the volume renders
    throughout: before any block (a zero volume), between blocks (the blocks
    not yet written read zero) and after volume_end, bit for bit against the
    oracle on the same partially written volume. Ragged extents, 3-D blocks
    of uneven sizes in shuffled order (block edges cut through bricks)."""
    full = cf.fbm_volume(48, 31, nthreads=8)[:41, :45, :37].copy()  # [D, H, W]
    D, H, W = full.shape
    rng = np.random.default_rng(5)
    zs, ys, xs = [0, 7, 20, 41], [0, 13, 30, 45], [0, 5, 22, 37]
    blocks = [((x0, y0, z0), (x1, y1, z1)) for z0, z1 in zip(zs[:-1], zs[1:])
              for y0, y1 in zip(ys[:-1], ys[1:]) for x0, x1 in zip(xs[:-1], xs[1:])]
    order = rng.permutation(len(blocks))
    R = 48
    gpu, cpu = make_pair(R, np.zeros((2, 2, 2), np.uint8), cf.tf_spectral(), ext=24.0, layout=layout)
    gpu.volume_begin(full.shape)
    part = np.zeros_like(full)
    cpu.volume = part.copy()
    mvp = cf.golden_mvp("orbit")
    seeds = cf.seed_stream(16, start=40)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0])
    k = 1

    def step(what):
        nonlocal k
        gpu.render(mvp, seeds[k])
        rgb, want = cpu.render(mvp, seeds[k])
        k += 1
        assert_photons_equal(gpu.read_photons(), cpu.photons, what)
        assert_rgba_equal(gpu.read_rgba16f(), want, what)
        assert_rgb32_equal(gpu.read_rgb(), rgb, what)

    step("no block yet")
    for j, bi in enumerate(order):
        (x0, y0, z0), (x1, y1, z1) = blocks[bi]
        gpu.volume_write_block((x0, y0, z0), full[z0:z1, y0:y1, x0:x1])
        part[z0:z1, y0:y1, x0:x1] = full[z0:z1, y0:y1, x0:x1]
        cpu.volume = part.copy()
        if j % 6 == 5:
            step(f"after {j + 1} of {len(blocks)} blocks")
    gpu.volume_end()
    assert np.array_equal(part, full)
    step("after volume_end")
    step("after volume_end, second pass")
    with pytest.raises(vptmcm.VptError, match="outside volume_begin"):
        gpu.volume_write_block((0, 0, 0), full[:1, :1, :1])
    gpu.close()


def test_blockwise_volume_ingest_equals_whole():
    """WebGPUVolume.readModality-style per-block writes land where they should."""
    vol = cf.fbm_volume(48, 99, nthreads=8)
    blocks = [((x, y, z), vol[z:z + 16, y:y + 24, x:x + 12])
              for z in range(0, 48, 16) for y in range(0, 48, 24) for x in range(0, 48, 12)]
    a = vptmcm.Renderer(32, device=0)
    a.volume_blocks(vol.shape, blocks)
    b, cpu = make_pair(32, vol, cf.tf_spectral())
    a.set_spectrum(cf.spectrum_buffer("12"))
    a.set_material_tf(cf.tf_spectral())
    a.set_light(*cf.light_default())
    a.set_params(extinction=32.0)
    mvp = cf.default_mvp_inverse()
    for r in (a, b):
        r.reset(mvp, 5)
        r.render(mvp, 6)
    cpu.reset(mvp, 5)
    cpu.render(mvp, 6)
    assert_photons_equal(b.read_photons(), cpu.photons, "whole volume")
    assert_photons_equal(a.read_photons(), cpu.photons, "block-wise volume")
    a.close()
    b.close()


@pytest.mark.parametrize("n", [256, 512])
def test_full_size_benchmark_config(n):
    """C2 (256^3 grey) and C3 (512^3 spectral, g = 0.702) at R = 512, bit-exact."""
    vol = cf.fbm_volume(n, 1234 if n == 256 else 512)
    tf = cf.tf_grey() if n == 256 else cf.tf_spectral()
    gpu, cpu = make_pair(512, vol, tf, ext=32.0)
    run_and_compare(gpu, cpu, cf.default_mvp_inverse(), cf.seed_stream(3, start=0),
                    f"C{2 if n == 256 else 3} R=512")
    gpu.close()


def test_properties_many_passes():
    """Size-independent properties over many passes at R = 512: sample counts are
    monotone, radiance is a running mean of values in [0, 5*max(spd)/255]."""
    vol = cf.fbm_volume(128, 512)
    gpu = vptmcm.Renderer(512, device=0)
    gpu.set_spectrum(cf.spectrum_buffer("12"))
    gpu.set_volume(vol)
    gpu.set_material_tf(cf.tf_spectral())
    gpu.set_light(*cf.light_default())
    gpu.set_params(extinction=32.0)
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, cf.seed_bits(0))
    gpu.render_passes(mvp, cf.seed_stream(20))
    a = gpu.read_photons()
    gpu.render_passes(mvp, cf.seed_stream(20, start=21))
    b = gpu.read_photons()
    assert (b[:, 7] >= a[:, 7]).all() and (b[:, 7] > 0).all()
    rad = b[:, 10:22].view(np.float32)
    assert np.isfinite(rad).all() and rad.min() >= 0 and rad.max() <= 5 * 100 / 255 + 1e-6
    gpu.close()


def test_composite_single_rank():
    """RCCL path with one rank: the composite equals the rank's own image."""
    gpu, _ = make_pair(64, cf.sphere_in_cube(64), cf.tf_spectral())
    gpu.comm_init(vptmcm.unique_id(), 1, 0)
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 1)
    for s in cf.seed_stream(3):
        gpu.render(mvp, s)
        gpu.allreduce_radiance()
    rgb, n = gpu.read_composite()
    img = gpu.read_rgb()  # the composite weights the fp32 image, not its f16 rounding
    ph = gpu.read_photons()
    assert np.array_equal(n.reshape(-1), ph[:, 7].astype(np.float32))
    m = n > 0
    np.testing.assert_allclose(rgb[m], img[m], rtol=3e-7, atol=0)  # (rgb*n)/n: <= 2 roundings

    def from_pack(pk):  # k_composite of one (rgb*n, n) buffer, in numpy (f32, correctly rounded)
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(pk[..., 3:] > 0, pk[..., :3] / pk[..., 3:], np.float32(0)).astype(np.float32)

    # the march wrote the all-reduced buffer itself (k_pack's values, no k_pack
    # launch): bit-exact against k_pack's buffer through the same division
    assert_rgb32_equal(rgb, from_pack(gpu.pack_radiance()), "fused pack vs k_pack")
    # a reset between the march and the all-reduce: k_pack packs the reset photons
    gpu.render_passes(mvp, cf.seed_stream(4, start=7))
    gpu.reset(mvp, 9)
    gpu.allreduce_radiance()
    rgb2, n2 = gpu.read_composite()
    assert (n2 == 0).all()  # a reset zeroes every sample count
    assert_rgb32_equal(rgb2, from_pack(gpu.pack_radiance()), "k_pack after a reset")
    gpu.barrier()
    v = gpu.allreduce_host([1.0, 2.0], op="max")
    assert list(v) == [1.0, 2.0]
    gpu.close()


def test_composite_single_rank_inline_and_side_stream():
    """VPTMCM_ALLREDUCE_INLINE (the all-reduce on the march stream) and the
    side-stream all-reduce, interleaved on one communicator, with and without
    a read between them, each also as a reduce-scatter (VPTMCM_ALLREDUCE_SHARDED,
    read through the all-gather; one rank: the whole frame is its shard): every
    composite read equals the division of k_pack's buffer of the frame it
    follows, bit for bit, and so the modes agree."""
    gpu, _ = make_pair(64, cf.sphere_in_cube(64), cf.tf_spectral())
    gpu.comm_init(vptmcm.unique_id(), 1, 0)
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 3)

    def from_pack(pk):
        with np.errstate(divide="ignore", invalid="ignore"):
            return np.where(pk[..., 3:] > 0, pk[..., :3] / pk[..., 3:], np.float32(0)).astype(np.float32)

    seeds = cf.seed_stream(40, start=50)
    modes = [(True, False), (False, True), (True, True), (True, False), (False, False), (False, True),
             (True, True), (False, False), (True, True)]
    for k, (inline, sharded) in enumerate(modes):
        gpu.render_passes(mvp, seeds[4 * k:4 * k + 4])
        gpu.allreduce_radiance(inline=inline, sharded=sharded)
        if k % 3 != 1:  # some composites are never read: the next one overtakes them
            rgb, n = gpu.read_composite()
            assert_rgb32_equal(rgb, from_pack(gpu.pack_radiance()),
                               f"composite {k} inline={inline} sharded={sharded}")
            assert np.array_equal(n.reshape(-1), gpu.read_photons()[:, 7].astype(np.float32))
    # a render() queued behind an inline all-reduce, then one more inline one
    gpu.allreduce_radiance(inline=True)
    gpu.render(mvp, seeds[-1])
    gpu.allreduce_radiance(inline=True, sharded=True)
    rgb, n = gpu.read_composite()
    assert_rgb32_equal(rgb, from_pack(gpu.pack_radiance()), "after a queued render")
    with pytest.raises(vptmcm.VptError, match="unknown flags"):
        gpu._ck(gpu.L.vptmcm_comm_allreduce_radiance_ex(gpu.h, 5))
    gpu.close()


@pytest.mark.parametrize("tfname,bands", [("spectral", [(0, 32), (32, 64)]),
                                          ("materials", [(0, 8), (8, 40), (40, 64)]),
                                          ("spectral", [(0, 24), (24, 56), (56, 60)])])
def test_mode_b_bands_bitexact(tfname, bands):
    """SURVEY 8e Mode B on the HIP path: band renderers (one per GPU in a real run;
    here several handles on one GPU) with the same seeds reproduce the full-frame
    renderer row for row — photons, rgba16f rows, and the fp32 image whose band
    sum (rows outside a band are zero) is the full image bit for bit. R = 60
    exercises a last band ending at R."""
    R = 60 if bands[-1][1] == 60 else 64
    tf = cf.tf_spectral() if tfname == "spectral" else cf.tf_materials(True)
    vol = cf.fbm_volume(48, 9, nthreads=8)
    full, _ = make_pair(R, vol, tf, ext=24.0)
    parts = []
    for y0, y1 in bands:
        g, _ = make_pair(R, vol, tf, ext=24.0)
        g.set_band(y0, y1)
        parts.append(g)
    mvp = cf.golden_mvp("orbit")
    seeds = cf.seed_stream(8, start=3)
    for g in [full] + parts:
        g.reset(mvp, seeds[0])
        for s in seeds[1:4]:
            g.render(mvp, s)
        g.render_passes(mvp, seeds[4:])
    want_ph, want_rgba, want_rgb = full.read_photons(), full.read_rgba16f(), full.read_rgb()
    acc = np.zeros_like(want_rgb)
    for (y0, y1), g in zip(bands, parts):
        ph = g.read_photons().reshape(R, R, -1)
        assert same_words(ph[y0:y1], want_ph.reshape(R, R, -1)[y0:y1]).all(), f"band {y0}:{y1} photons"
        assert np.array_equal(g.read_rgba16f()[y0:y1], want_rgba[y0:y1]), f"band {y0}:{y1} image"
        rgb = g.read_rgb()
        assert not rgb[:y0].any() and not rgb[y1:].any(), "rows outside the band stay zero"
        acc += rgb
    assert same_words(acc.view(np.uint32), want_rgb.view(np.uint32)).all(), "band composite"
    with pytest.raises(vptmcm.VptError):
        parts[0].set_band(4, 16)  # not a multiple of 8
    for g in [full] + parts:
        g.close()


def test_mode_b_gather_single_rank():
    """vptmcm_comm_gather_bands over RCCL with one rank: the rank's own fp32 image."""
    gpu, _ = make_pair(64, cf.sphere_in_cube(64), cf.tf_spectral())
    gpu.comm_init(vptmcm.unique_id(), 1, 0)
    gpu.set_band(16, 48)
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 5)
    gpu.render_passes(mvp, cf.seed_stream(4))
    img = gpu.read_rgb()
    assert not img[:16].any() and not img[48:].any()
    # one rank's band must cover the frame: rows [0, 16) and [48, 64) are in no band
    with pytest.raises(vptmcm.VptError, match="covered by 0 ranks") as e:
        gpu.gather_bands()
    assert e.value.code == vptmcm.ECOMM
    gpu.set_band(0, 64)  # the communicator survives a coverage error
    assert np.array_equal(gpu.gather_bands().view(np.uint32), img.view(np.uint32))
    gpu.close()


def test_comm_peer_never_joins_fails_before_rccl():
    """A two-rank job whose second rank never arrives: rank
    0 fails in the all-ranks-present rendezvous with ECOMM after the bound,
    before any RCCL call (RCCL 2.27.7's init cannot be bounded from outside:
    it does not return while its bootstrap waits), so no RCCL
    thread is started or left behind: the process's thread count is unchanged,
    and the handle stays usable without a communicator."""
    import os
    import time

    from vptmcm import rendezvous

    def threads():
        return len(os.listdir("/proc/self/task"))

    gpu, _ = make_pair(32, cf.sphere_in_cube(32), cf.tf_spectral())
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 3)
    gpu.synchronize()
    before = threads()
    key = f"never-joins-{os.getpid()}"
    t0 = time.monotonic()
    with pytest.raises(rendezvous.RendezvousError) as e:
        rendezvous.join(0, 2, key=key, timeout_s=3.0)
    took = time.monotonic() - t0
    rendezvous.cleanup(key, 2)
    assert e.value.code == vptmcm.ECOMM and 3.0 <= took < 30.0, (str(e.value), took)
    assert threads() == before, (before, threads())
    with pytest.raises(vptmcm.VptError, match="no communicator"):
        gpu.barrier()
    gpu.render_passes(mvp, cf.seed_stream(2))
    gpu.synchronize()
    assert threads() == before
    gpu.close()


def test_kernel_timing_counts_launches():
    """render_passes fuses up to 32 passes per march launch."""
    gpu, _ = make_pair(64, cf.sphere_in_cube(64), cf.tf_spectral())
    mvp = cf.default_mvp_inverse()
    gpu.reset(mvp, 1)
    gpu.enable_kernel_timing(True)
    gpu.render_passes(mvp, cf.seed_stream(5))
    gpu.render_passes(mvp, cf.seed_stream(40, start=5))
    ms, n = gpu.kernel_time()
    assert n == 3 and ms > 0  # 5 | 32 + 8
    gpu.close()


@pytest.mark.parametrize("layout", LAYOUTS)
@pytest.mark.parametrize("R", [64, 72])
def test_fused_passes_bitexact(layout, R):
    """render_passes keeps the photon state in registers across the passes of
    one launch (32 per launch here: 37 = 32 + 5); photon state and the last
    pass's image equal the oracle's after the same passes one by one."""
    gpu, cpu = make_pair(R, cf.two_spheres(48), cf.tf_materials(True), ext=24.0, layout=layout)
    mvp = cf.golden_mvp("orbit")
    seeds = cf.seed_stream(38, start=3)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0])
    gpu.render_passes(mvp, seeds[1:])
    for s in seeds[1:]:
        _, want = cpu.render(mvp, s)
    assert_photons_equal(gpu.read_photons(), cpu.photons, f"fused R={R}")
    assert_rgba_equal(gpu.read_rgba16f(), want, f"fused R={R}")
    gpu.close()


def test_lazily_fused_render_calls():
    """render() queues passes and launches them fused when anything else is
    called (here: 40 renders = 32 + 8 with a matrix change in between, a
    parameter setter and reads): photons and image equal the oracle's passes
    one by one, and the launch count shows the fusion happened."""
    gpu, cpu = make_pair(64, cf.two_spheres(48), cf.tf_materials(True), ext=24.0)
    m1, m2 = cf.golden_mvp("orbit"), cf.golden_mvp("near")
    seeds = cf.seed_stream(60, start=11)
    gpu.reset(m1, seeds[0])
    cpu.reset(m1, seeds[0])
    gpu.enable_kernel_timing(True)
    for s in seeds[1:41]:
        gpu.render(m1, s)
        cpu.render(m1, s)
    for s in seeds[41:47]:
        gpu.render(m2, s)
        _, want = cpu.render(m2, s)
    ms, n = gpu.kernel_time()  # flushes the queue
    assert n == 3, n  # 32 + 8 passes with m1, 6 with m2
    assert_photons_equal(gpu.read_photons(), cpu.photons, "lazy fused")
    assert_rgba_equal(gpu.read_rgba16f(), want, "lazy fused")
    gpu.render(m2, seeds[47])
    cpu.render(m2, seeds[47])
    gpu.set_params(extinction=12.0, bounces=8, steps=8)  # flushes with the old params
    cpu.params.update(extinction=12.0)
    for s in seeds[48:52]:
        gpu.render(m2, s)
        _, want = cpu.render(m2, s)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "lazy fused after setter")
    assert_rgba_equal(gpu.read_rgba16f(), want, "lazy fused after setter")
    gpu.close()


def test_schedule_and_fusion_knobs_agree(monkeypatch):
    """The tile schedule (variant bit 1 = raster mapping) and pass fusion
    (variant bit 2 = one launch per pass) only change which wave runs a tile and
    how launches are cut: all four combinations give identical bits."""
    vol, tf = cf.fbm_volume(64, 9), cf.tf_spectral()
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(12, start=50)
    out = []
    for variant in (0, 2, 4, 6):
        monkeypatch.setenv("VPTMCM_MARCH_VARIANT", str(variant))
        gpu, _ = make_pair(128, vol, tf, ext=32.0)
        gpu.reset(mvp, seeds[0])
        gpu.render_passes(mvp, seeds[1:6])
        gpu.render_passes(mvp, seeds[6:])
        out.append((gpu.read_photons(), gpu.read_rgba16f()))
        gpu.close()
    for ph, img in out[1:]:
        assert np.array_equal(ph, out[0][0]) and np.array_equal(img, out[0][1])


def test_render_without_volume_fails_loudly():
    gpu = vptmcm.Renderer(16, device=0)
    with pytest.raises(vptmcm.VptError, match="no volume"):
        gpu.render(cf.default_mvp_inverse(), 1)
    with pytest.raises(vptmcm.VptError, match="n_bins"):
        gpu.set_spectrum(np.float32([13.0] + [0] * 63))
    gpu.close()


def _poses():
    import json
    return list(json.loads((cf.GOLDEN / "mvp_inverse.json").read_text())["cameras"])


@pytest.mark.parametrize("camera", _poses())
def test_fused_full_size_robust_background(camera):
    """R = 512 with 16 fused passes: background tiles run the robust-miss path
    (no distance/advance/bounds/slab per step, start point materialised once
    per launch); photon state and image equal the oracle's pass-by-pass run."""
    mvp = cf.golden_mvp(camera)
    gpu, cpu = make_pair(512, cf.fbm_volume(128, 77), cf.tf_spectral(), ext=32.0)
    seeds = cf.seed_stream(17, start=100)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:])
    for s in seeds[1:]:
        _, want = cpu.render(mvp, s, nthreads=16)
    assert_photons_equal(gpu.read_photons(), cpu.photons, f"fused R=512 {camera}")
    assert_rgba_equal(gpu.read_rgba16f(), want, f"fused R=512 {camera}")
    gpu.close()


def test_camera_change_without_reset():
    """Photons carried into a launch from another camera (no reset between):
    the robust path only engages after a lane's first reset under the current
    matrix, so the result still equals the oracle's."""
    other = [n for n in _poses() if n != "default"]
    mvps = [cf.default_mvp_inverse(), cf.golden_mvp(other[0])]
    gpu, cpu = make_pair(256, cf.fbm_volume(64, 5), cf.tf_spectral(), ext=8.0)
    seeds = cf.seed_stream(13, start=7)
    gpu.reset(mvps[0], seeds[0])
    cpu.reset(mvps[0], seeds[0], nthreads=16)
    gpu.render_passes(mvps[0], seeds[1:7])
    gpu.render_passes(mvps[-1], seeds[7:])
    for k, s in enumerate(seeds[1:], 1):
        _, want = cpu.render(mvps[0] if k < 7 else mvps[-1], s, nthreads=16)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "camera change")
    assert_rgba_equal(gpu.read_rgba16f(), want, "camera change")
    gpu.close()


def test_schedule_changes_every_launch(monkeypatch):
    """A wave slot starts loading the photon state of the tile it ran last
    launch before its schedule is known (TileSched::prev) and reloads when the
    schedule moved it: one-pass launches that alternate between two cameras
    (different volume tiles every launch, so most slots change tile), then a
    band change on the same handle, equal the oracle pass by pass."""
    monkeypatch.setenv("VPTMCM_MARCH_VARIANT", "4")  # one launch per pass
    mvps = [cf.default_mvp_inverse(), cf.golden_mvp("near")]
    gpu, cpu = make_pair(256, cf.fbm_volume(64, 21), cf.tf_spectral(), ext=16.0)
    seeds = cf.seed_stream(12, start=31)
    gpu.reset(mvps[0], seeds[0])
    cpu.reset(mvps[0], seeds[0], nthreads=16)
    for k, s in enumerate(seeds[1:9]):
        gpu.render_passes(mvps[k & 1], [s])
        _, want = cpu.render(mvps[k & 1], s, nthreads=16)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "alternating schedule")
    assert_rgba_equal(gpu.read_rgba16f(), want, "alternating schedule")
    gpu.set_band(64, 192)
    ref = vptmcm.Renderer(256, device=0)  # the same band on a fresh handle (no previous schedule)
    ref.set_volume(cf.fbm_volume(64, 21))
    ref.set_material_tf(cf.tf_spectral())
    spd, ldir = cf.light_default()
    ref.set_light(spd, ldir)
    ref.set_spectrum(cf.spectrum_buffer("12"))
    ref.set_params(extinction=16.0, bounces=8, steps=8)
    ref.write_photons(gpu.read_photons())
    ref.set_band(64, 192)
    for s in seeds[9:]:
        gpu.render_passes(mvps[0], [s])
        ref.render_passes(mvps[0], [s])
    assert np.array_equal(gpu.read_photons(), ref.read_photons())
    assert np.array_equal(gpu.read_rgba16f()[64:192], ref.read_rgba16f()[64:192])
    gpu.close()
    ref.close()


def _xcd_unswizzle(lb: int, G: int) -> int:
    """Inverse of march.h xcd_swizzle: the hardware block of swizzled block lb."""
    if G % 8:
        return lb
    x, r = divmod(lb, G // 8)
    return r * 8 + x


def _expected_schedule(table: np.ndarray, n_tiles: int, xcd_by_xcd: bool = False) -> np.ndarray:
    """schedule_tile's deal (kernels.hip), restated: tiles ordered [volume
    tiles, background tiles], each class ascending; slot q = k*4G + lb*4 + j
    goes to wave 4j + ((k + j) & 3) of hardware block lb (consecutive blocks
    rotate over the XCDs), or of block unswizzle(lb) with round 2's XCD-by-XCD
    order (variant bit 7). The volume class is taken from the table's own bit 31."""
    G = table.size // 16
    used = table != 0xFFFFFFFF
    words = table[used]
    tiles = words & 0x1FFFFFFF
    vol = np.zeros(n_tiles, bool)
    vol[tiles[(words >> 31) == 1]] = True
    nv = int(vol.sum())
    slots = {}
    for q, t in enumerate(np.flatnonzero(vol)):
        slots[int(t)] = q
    for r, t in enumerate(np.flatnonzero(~vol)):
        slots[int(t)] = nv + r
    exp = np.full(table.size, 0xFFFFFFFF, np.uint32)
    for t, q in slots.items():
        k, rem = divmod(q, 4 * G)
        lb, j = divmod(rem, 4)
        b = _xcd_unswizzle(lb, G) if xcd_by_xcd else lb
        exp[b * 16 + 4 * j + ((k + j) & 3)] = t | (int(vol[t]) << 31)
    return exp


@pytest.mark.parametrize("R,variant", [(256, "0"), (512, "0"), (512, "128"), (1024, "0")])
def test_tile_schedule_is_the_latin_square_deal(R, variant, monkeypatch):
    """N2, checked directly: after each launch every tile ran on exactly one
    wave slot, volume tiles first, dealt over the slots exactly as
    schedule_tile's ballot / prefix scan intends (vptmcm_debug_schedule), in
    the XCD round-robin slot order and in round 2's XCD-by-XCD one (variant
    bit 7); a camera change re-deals it."""
    monkeypatch.setenv("VPTMCM_MARCH_VARIANT", variant)
    gpu = vptmcm.Renderer(R, device=0)
    assert (gpu.debug_schedule() == 0xFFFFFFFF).all()  # fresh handle: no launch yet
    gpu.set_volume(cf.fbm_volume(128, 77))
    gpu.set_material_tf(cf.tf_spectral())
    spd, ldir = cf.light_default()
    gpu.set_light(spd, ldir)
    gpu.set_spectrum(cf.spectrum_buffer("12"))
    gpu.set_params(extinction=32.0, bounces=8, steps=8)
    n_tiles = (R // 8) ** 2
    seeds = cf.seed_stream(12, start=3)
    gpu.reset(cf.default_mvp_inverse(), seeds[0])
    vset = []
    for k, mvp in enumerate([cf.default_mvp_inverse()] * 3 + [cf.golden_mvp("near")] * 2):
        gpu.render_passes(mvp, seeds[1 + 2 * k:3 + 2 * k])
        tab = gpu.debug_schedule()
        used = tab[tab != 0xFFFFFFFF]
        assert np.array_equal(np.sort(used & 0x1FFFFFFF), np.arange(n_tiles)), f"launch {k}: not a permutation"
        assert np.array_equal(tab, _expected_schedule(tab, n_tiles, variant == "128")), \
            f"launch {k}: deal differs"
        vset.append(frozenset((used[(used >> 31) == 1] & 0x1FFFFFFF).tolist()))
    assert not vset[0] and 0 < len(vset[1]) < n_tiles  # flags start clear, then a volume class
    assert vset[4] != vset[2]  # the second camera's tiles, one launch after it took over
    gpu.close()


def test_tiny_resolutions_and_empty_volume():
    """R = 1, 2, 3 (one partial tile, pixel centres on the screen axes for odd R:
    the near point is then not hoisted) and an all-zero volume."""
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(4, start=5)
    for R in (1, 2, 3):
        gpu, cpu = make_pair(R, cf.sphere_in_cube(16), cf.tf_spectral(), ext=8.0)
        run_and_compare(gpu, cpu, mvp, seeds, f"R={R}")
        gpu.close()
    gpu, cpu = make_pair(16, np.zeros((8, 8, 8), np.uint8), cf.tf_spectral(), ext=8.0)
    run_and_compare(gpu, cpu, mvp, seeds, "empty volume")
    gpu.close()


def test_large_frame_rows_against_oracle():
    """R = 2048 (65536 tiles: the raster tile mapping, 4.2 M photons): a band of
    rows through the cube and the image edge, checked against the oracle's
    row-restricted run after two fused passes."""
    R = 2048
    vol = cf.fbm_volume(128, 99)
    gpu, cpu = make_pair(R, vol, cf.tf_spectral(), ext=32.0)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(3, start=9)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:])
    for s in seeds[1:]:
        _, want = cpu.render(mvp, s, nthreads=16, rows=(1000, 1040))
    got = gpu.read_photons().reshape(R, R, -1)
    exp = cpu.photons.reshape(R, R, -1)
    for y0, y1 in ((1000, 1040),):
        assert_photons_equal(got[y0:y1].reshape(-1, got.shape[-1]), exp[y0:y1].reshape(-1, exp.shape[-1]),
                             f"R=2048 rows {y0}:{y1}")
        assert_rgba_equal(gpu.read_rgba16f()[y0:y1], want[y0:y1], f"R=2048 rows {y0}:{y1}")
    gpu.close()


def test_multi_chunk_schedule_rows_against_oracle():
    """R = 1024 (16384 tiles: the largest frame with the balanced schedule, whose
    ballot / prefix scan runs in four 4096-tile chunks after a counting pass): a
    band of rows through the cube, checked against the oracle after a one-pass
    launch (flags all clear) and a fused launch dealt from the first one's flags."""
    R = 1024
    gpu, cpu = make_pair(R, cf.fbm_volume(128, 98), cf.tf_spectral(), ext=32.0)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(5, start=21)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:2])
    gpu.render_passes(mvp, seeds[2:])
    rows = (480, 528)
    for s in seeds[1:]:
        _, want = cpu.render(mvp, s, nthreads=16, rows=rows)
    got = gpu.read_photons().reshape(R, R, -1)[rows[0]:rows[1]]
    exp = cpu.photons.reshape(R, R, -1)[rows[0]:rows[1]]
    assert_photons_equal(got.reshape(-1, got.shape[-1]), exp.reshape(-1, exp.shape[-1]), "R=1024 rows")
    assert_rgba_equal(gpu.read_rgba16f()[rows[0]:rows[1]], want[rows[0]:rows[1]], "R=1024 rows")
    tab = gpu.debug_schedule()
    assert int((tab[tab != 0xFFFFFFFF] >> 31).sum()) > 0  # the second launch had a volume class
    gpu.close()


def _oracle_pack(cpu, rgb32):
    """(rgb*n, n) per pixel in f32, as k_pack forms it (n = photon sample count)."""
    n = cpu.photons[:, 7].astype(np.float32).reshape(cpu.R, cpu.R)
    return np.concatenate([rgb32 * n[..., None], n[..., None]], axis=-1).astype(np.float32)


def test_c4_two_replica_composite_bitexact():
    """C4's composite on one GPU, without RCCL: two replicas with the rank seed
    streams seed_bits(k, 0) and seed_bits(k, 1), each packed by k_pack from its
    fp32 image, summed on the host; bit-exact against two oracle replicas
    composited the same way (f32 sum of two terms is order-free; the composite
    divides by the summed count as vptmcm_comm_read_composite does)."""
    R, passes = 128, 6
    vol, tf, mvp = cf.fbm_volume(96, 4, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    packs, wants = [], []
    for rank in (0, 1):
        gpu, cpu = make_pair(R, vol, tf, ext=32.0)
        seeds = cf.seed_stream(passes + 1, start=0, rank=rank)
        gpu.reset(mvp, seeds[0])
        cpu.reset(mvp, seeds[0], nthreads=16)
        gpu.render_passes(mvp, seeds[1:])
        for s in seeds[1:]:
            rgb, _ = cpu.render(mvp, s, nthreads=16)
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"replica {rank}")
        got = gpu.pack_radiance()
        want = _oracle_pack(cpu, rgb)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"k_pack replica {rank}"
        packs.append(got)
        wants.append(want)
        gpu.close()
    assert not np.array_equal(packs[0], packs[1]), "rank seed streams must differ"
    tot, wtot = packs[0] + packs[1], wants[0] + wants[1]
    assert np.array_equal(tot.view(np.uint32), wtot.view(np.uint32))
    n = tot[..., 3]
    comp = np.where(n[..., None] > 0, tot[..., :3] / np.where(n > 0, n, 1)[..., None], 0)
    assert np.isfinite(comp).all() and (n > 0).mean() > 0.99


def test_c4_full_size_eight_replica_packs():
    """C4 at its own size on one GPU: the C3 workload (512^3 fBm, spectral TF,
    R = 512, S = 8, extinction 32) as the eight replicas of an 8-GPU job, i.e.
    the rank seed streams seed_bits(k, 0..7), one after the other on one
    renderer. Every replica's photons and its k_pack (rgb*n, n) buffer are
    bit-exact against the oracle. The 8-term composite is exact per replica
    only: RCCL's summation order is its own, so the f32 sum is held to the f64
    sum within 8 ulp of the
    summed magnitudes."""
    R, passes, world = 512, 2, 8
    vol, tf, mvp = cf.fbm_volume(512, 512, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    gpu, cpu = make_pair(R, vol, tf, ext=32.0)
    packs = []
    for rank in range(world):
        seeds = cf.seed_stream(passes + 1, start=0, rank=rank)
        gpu.reset(mvp, seeds[0])
        cpu.reset(mvp, seeds[0], nthreads=16)
        gpu.render_passes(mvp, seeds[1:])
        for s in seeds[1:]:
            rgb, _ = cpu.render(mvp, s, nthreads=16)
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"C4 replica {rank}")
        got = gpu.pack_radiance()
        assert np.array_equal(got.view(np.uint32), _oracle_pack(cpu, rgb).view(np.uint32)), \
            f"C4 k_pack replica {rank}"
        packs.append(got)
    gpu.close()
    assert len({p.tobytes() for p in packs}) == world, "rank seed streams must differ"
    tot32 = np.zeros_like(packs[0])
    for p in packs:
        tot32 += p
    tot64 = np.sum([p.astype(np.float64) for p in packs], axis=0)
    mag = np.sum([np.abs(p.astype(np.float64)) for p in packs], axis=0)
    assert (np.abs(tot32 - tot64) <= 8 * 2.0 ** -24 * mag).all()  # any summation order
    n = tot32[..., 3]
    assert (n == tot64[..., 3]).all()  # sample counts are small integers: exact in f32
    comp = tot32[..., :3] / np.where(n > 0, n, 1)[..., None]
    assert np.isfinite(comp).all() and (n > 0).mean() > 0.99


@pytest.mark.parametrize("layout", [vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_BRICK8])
def test_wide_gather_template_bitexact(layout, monkeypatch):
    """The 64-bit-offset CORNER8 / BRICK8 gathers (selected for cell arrays >= 4
    GiB, e.g. C5's 1024^3) forced on a small volume (variant bit 3): bit-exact."""
    monkeypatch.setenv("VPTMCM_MARCH_VARIANT", "8")
    gpu, cpu = make_pair(96, cf.fbm_volume(72, 21, nthreads=8), cf.tf_materials(True), ext=24.0,
                         layout=layout)
    run_and_compare(gpu, cpu, cf.golden_mvp("orbit"), cf.seed_stream(4, start=2), "wide gather")
    gpu.close()


@pytest.mark.parametrize("shape", [(37, 50, 23), (5, 4, 130), (1, 1, 1)])
def test_brick8_ragged_volume_bitexact(shape):
    """BRICK8 on volumes whose cell grid (W+1, H+1, D+1) is not a whole number of
    4x4x4 bricks (padding bricks, a 1-voxel volume): bit-exact against the oracle."""
    rng = np.random.default_rng(sum(shape))
    vol = rng.integers(0, 256, size=shape[::-1], dtype=np.uint8)
    gpu, cpu = make_pair(64, vol, cf.tf_materials(True), ext=20.0, layout=vptmcm.LAYOUT_BRICK8)
    run_and_compare(gpu, cpu, cf.golden_mvp("orbit_tilted"), cf.seed_stream(3, start=9),
                    f"brick8 {shape}")
    gpu.close()


@pytest.mark.parametrize("layout,tpl", [(vptmcm.LAYOUT_CORNER8, 2), (vptmcm.LAYOUT_COLUMN4, 6)])
def test_c5_1024_volume_streamed_rows_against_oracle(layout, tpl):
    """C5 on one GPU: the 1024^3 fBm volume (seed 1024) streamed into HBM in
    64-slice blocks (WebGPUVolume.readModality's per-placement upload), CORNER8
    cells > 4 GiB (the 64-bit gather template); R = 512, two fused passes; a
    band of rows through the cube is bit-exact against the oracle's
    row-restricted run, and the whole frame satisfies the running-mean bounds."""
    n, R = 1024, 512
    vol = cf.fbm_volume(n, 1024)
    gpu = vptmcm.Renderer(R, device=0, layout=layout)
    gpu.volume_blocks(vol.shape, (((0, 0, z), vol[z:z + 64]) for z in range(0, n, 64)))
    cpu = orc.Oracle(R)
    spec, tf = cf.spectrum_buffer("12"), cf.tf_spectral()
    spd, ld = cf.light_default()
    for r in (gpu, cpu):
        r.set_spectrum(spec)
    gpu.set_material_tf(tf)
    gpu.set_light(spd, ld)
    gpu.set_params(extinction=32.0, bounces=8, steps=8)
    cpu.volume, cpu.tf, cpu.light, cpu.light_dir = vol, tf, spd, ld
    cpu.params.update(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(3, start=40)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:])
    assert gpu.last_launch()["tpl"] == tpl  # cells over 4 GiB: the 64-bit gather
    rows = (224, 264)
    for s in seeds[1:]:
        rgb, want = cpu.render(mvp, s, nthreads=16, rows=rows)
    y0, y1 = rows
    got = gpu.read_photons().reshape(R, R, -1)
    exp = cpu.photons.reshape(R, R, -1)
    assert_photons_equal(got[y0:y1].reshape(-1, got.shape[-1]), exp[y0:y1].reshape(-1, exp.shape[-1]),
                         "C5 rows")
    assert_rgba_equal(gpu.read_rgba16f()[y0:y1], want[y0:y1], "C5 rows")
    assert_rgb32_equal(gpu.read_rgb()[y0:y1], rgb[y0:y1], "C5 rows fp32")
    allp = got.reshape(R * R, -1)
    rad = allp[:, 10:22].view(np.float32)
    # a photon that scattered or null-collided through all 16 steps has no
    # sample yet (samples 0, bins still the reset's 1.0)
    smp = allp[:, 7]
    assert (smp <= 16).all() and (smp >= 1).mean() > 0.9 and np.isfinite(rad).all()
    assert rad.min() >= 0 and rad[smp >= 1].max() <= 5 * 100 / 255 + 1e-6
    assert (rad[smp == 0] == 1.0).all()
    gpu.close()


@pytest.mark.parametrize("layout,tpl", [(vptmcm.LAYOUT_COLUMN4, 5), (vptmcm.LAYOUT_CORNER8, 1)])
@pytest.mark.parametrize("dark", ["0", "1"])
def test_c3_driver_shaped_launch_bitexact(dark, layout, tpl, monkeypatch):
    """The benchmarked launch shape itself: BASELINE C3
    (512^3 fBm seed 512, spectral TF, R = 512, S = 8, 12 bins, extinction 32,
    default camera) from a reset, the driver's 5 warm-up passes as one launch,
    then its timed `--steps 20` region as ONE 20-pass fused launch (the FAST
    MODE 2 kernel on COLUMN4, the bench's default layout, and on CORNER8), with the
    bench's own seed stream: photons, the
    fp32 image and the rgba16f image bit-exact against the oracle, with the
    dark-background chain (the default: background waves the light never
    reaches run the draw chain alone) and without it (VPTMCM_DARK=0)."""
    monkeypatch.setenv("VPTMCM_DARK", dark)
    R, S = 512, 8
    vol, tf, mvp = cf.fbm_volume(512, 512, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    gpu, cpu = make_pair(R, vol, tf, ext=32.0, steps=S, layout=layout)
    seeds = cf.seed_stream(1 + 5 + 20, start=0, rank=0)  # bench.py's stream at N = 1
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    gpu.render_passes(mvp, seeds[1:6])
    gpu.render_passes(mvp, seeds[6:26])
    info = gpu.last_launch()
    assert (info["passes"], info["mode"], info["tpl"], info["spec"]) == (20, 2, tpl, True), info
    for s in seeds[1:]:
        rgb, want = cpu.render(mvp, s, nthreads=16)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "C3 20-pass launch")
    assert_rgb32_equal(gpu.read_rgb(), rgb, "C3 20-pass launch")
    assert_rgba_equal(gpu.read_rgba16f(), want, "C3 20-pass launch")
    gpu.close()


def test_c3_bench_settled_state_driver_launch_rows_bitexact():
    """The state the benchmark actually times: bench.py
    resets, then runs clock-settling launches of 32 passes with a seed stream
    of their own (cf.seed_stream(32, start=1 << 20), replayed launch after
    launch, ~10,240 passes in its 150 ms), then the driver's 5 warm-up passes
    and its timed 20-pass launch. Here the same sequence on C3 at full size with
    exactly 320 settling launches (10,240 passes: photons holding ~10^4
    samples, the large-n running-mean division), then 5 + 20: the photons and
    both images of a 16-row band through the cube are bit-exact against the
    oracle's row-restricted run of all 10,265 passes (photons are independent
    per pixel, so a band of the full frame is the band's own run), and the
    whole frame's sample counts are those of the settled state."""
    R, S = 512, 8
    vol, tf, mvp = cf.fbm_volume(512, 512, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    gpu, cpu = make_pair(R, vol, tf, ext=32.0, steps=S, layout=vptmcm.LAYOUT_COLUMN4)  # the bench's layout
    seeds = cf.seed_stream(1 + 5 + 20, start=0, rank=0)  # bench.py's stream at N = 1
    sseeds = cf.seed_stream(32, start=1 << 20, rank=0)    # bench.py's clock-settling seeds
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    for _ in range(320):
        gpu.render_passes(mvp, sseeds)
    gpu.render_passes(mvp, seeds[1:6])
    gpu.render_passes(mvp, seeds[6:26])
    info = gpu.last_launch()
    assert (info["passes"], info["mode"], info["tpl"], info["spec"]) == (20, 2, 5, True), info
    rows = (248, 264)
    for _ in range(320):
        for s in sseeds:
            cpu.render(mvp, s, nthreads=16, rows=rows)
    for s in seeds[1:]:
        rgb, want = cpu.render(mvp, s, nthreads=16, rows=rows)
    y0, y1 = rows
    got = gpu.read_photons().reshape(R, R, -1)
    exp = cpu.photons.reshape(R, R, -1)
    assert_photons_equal(got[y0:y1].reshape(-1, got.shape[-1]), exp[y0:y1].reshape(-1, exp.shape[-1]),
                         "C3 settled, 20-pass launch")
    assert_rgb32_equal(gpu.read_rgb()[y0:y1], rgb[y0:y1], "C3 settled, 20-pass launch")
    assert_rgba_equal(gpu.read_rgba16f()[y0:y1], want[y0:y1], "C3 settled, 20-pass launch")
    smp = got.reshape(R * R, -1)[:, 7]
    band = got[y0:y1, :, 7]
    assert smp.max() > 10000 and np.median(band) > 1000, (smp.max(), np.median(band))
    gpu.close()


def test_c3_bench_default_region_rows_bitexact():
    """The state the default bench line times (`python bench.py`: 10,240
    clock-settling passes, 4,096 warm-up passes, then the 1,024 timed passes,
    all in 32-pass launches): a 16-row band through the cube bit-exact against
    the oracle's row-restricted run of all 15,361 passes."""
    R, S = 512, 8
    vol, tf, mvp = cf.fbm_volume(512, 512, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    gpu, cpu = make_pair(R, vol, tf, ext=32.0, steps=S, layout=vptmcm.LAYOUT_COLUMN4)
    W, K = 4096, 1024
    seeds = cf.seed_stream(1 + W + K, start=0, rank=0)
    sseeds = cf.seed_stream(32, start=1 << 20, rank=0)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    for _ in range(320):
        gpu.render_passes(mvp, sseeds)
    gpu.render_passes(mvp, seeds[1:1 + W])
    gpu.render_passes(mvp, seeds[1 + W:])
    info = gpu.last_launch()
    assert (info["passes"], info["mode"], info["tpl"]) == (32, 2, 5), info
    rows = (256, 272)
    for _ in range(320):
        for s in sseeds:
            cpu.render(mvp, s, nthreads=16, rows=rows)
    for s in seeds[1:]:
        rgb, want = cpu.render(mvp, s, nthreads=16, rows=rows)
    y0, y1 = rows
    got = gpu.read_photons().reshape(R, R, -1)
    exp = cpu.photons.reshape(R, R, -1)
    assert_photons_equal(got[y0:y1].reshape(-1, got.shape[-1]), exp[y0:y1].reshape(-1, exp.shape[-1]),
                         "C3 default bench region")
    assert_rgb32_equal(gpu.read_rgb()[y0:y1], rgb[y0:y1], "C3 default bench region")
    assert_rgba_equal(gpu.read_rgba16f()[y0:y1], want[y0:y1], "C3 default bench region")
    assert np.median(got[y0:y1, :, 7]) > 1500
    gpu.close()


@pytest.mark.parametrize("layout", [vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_BRICK8])
def test_queued_renders_matrix_change_and_inputs(layout):
    """render() calls queue passes that launch as fused marches: a render()
    with another camera launches the queued passes with their own matrix first,
    an input change (set_params) launches them with the old inputs, and a full
    queue of 32 launches on its own; the UI-like TF with uneven bins (MODE 6)
    too. Oracle: the same passes in order."""
    R = 128
    vol, mvp1, mvp2 = cf.fbm_volume(96, 17, nthreads=8), cf.golden_mvp("orbit"), cf.default_mvp_inverse()
    for tf, spec in ((cf.tf_spectral(), "12"), (cf.tf_materials(True), "8_uneven")):
        gpu, cpu = make_pair(R, vol, tf, spec=spec, ext=24.0, layout=layout)
        seeds = cf.seed_stream(120, start=5)
        gpu.reset(mvp1, seeds[0])
        cpu.reset(mvp1, seeds[0], nthreads=16)
        k = 1
        for _ in range(40):  # one full queue with camera 1, 8 queued
            gpu.render(mvp1, seeds[k])
            cpu.render(mvp1, seeds[k], nthreads=16)
            k += 1
        for _ in range(40):  # camera 2: the queued camera-1 passes launch first
            gpu.render(mvp2, seeds[k])
            cpu.render(mvp2, seeds[k], nthreads=16)
            k += 1
        gpu.set_params(extinction=12.0, bounces=8, steps=8)  # launches the queue with extinction 24
        cpu.params.update(extinction=12.0)
        for _ in range(36):
            gpu.render(mvp2, seeds[k])
            rgb, want = cpu.render(mvp2, seeds[k], nthreads=16)
            k += 1
        assert_photons_equal(gpu.read_photons(), cpu.photons, f"queued renders, camera change, {spec}")
        assert_rgba_equal(gpu.read_rgba16f(), want, f"queued renders, camera change, {spec}")
        assert_rgb32_equal(gpu.read_rgb(), rgb, f"queued renders, camera change, {spec}")
        gpu.close()


def test_screen_filling_volume_schedule():
    """Every tile in the volume (the 'near' camera fills the screen: 256 volume
    tiles on 64 SIMDs, so no SIMD holds a lone volume wave): every tile has
    exactly one wave slot of the deal, and photons and images stay bit-exact."""
    R = 128
    gpu, cpu = make_pair(R, cf.fbm_volume(96, 19, nthreads=8), cf.tf_spectral(), ext=24.0)
    mvp = cf.golden_mvp("near")
    seeds = cf.seed_stream(70, start=11)
    gpu.reset(mvp, seeds[0])
    cpu.reset(mvp, seeds[0], nthreads=16)
    for s in seeds[1:]:
        gpu.render(mvp, s)
        rgb, want = cpu.render(mvp, s, nthreads=16)
    assert_photons_equal(gpu.read_photons(), cpu.photons, "screen-filling volume")
    assert_rgba_equal(gpu.read_rgba16f(), want, "screen-filling volume")
    assert_rgb32_equal(gpu.read_rgb(), rgb, "screen-filling volume")
    slots = gpu.debug_schedule()
    dealt = slots[slots != 0xFFFFFFFF]
    tiles = dealt & 0x1FFFFFFF
    assert len(tiles) == (R // 8) ** 2 and len(np.unique(tiles)) == len(tiles), "one slot per tile"
    assert ((dealt >> 31) == 1).all(), "every tile entered the volume"
    gpu.close()


def test_dark_background_light_and_camera_changes(monkeypatch):
    """The dark-background chain where its conditions change between launches without a
    reset: the light flips from +x to -x (lit pixels' bins are no longer zero,
    dark ones become lit), then the camera moves (the stored photons come from
    the old camera: the launch's first step decides). Every launch bit-exact
    against the oracle, photons and both images."""
    monkeypatch.setenv("VPTMCM_DARK", "1")
    R = 128
    vol, tf = cf.fbm_volume(96, 21, nthreads=8), cf.tf_spectral()
    gpu, cpu = make_pair(R, vol, tf, ext=24.0)
    spd = np.full(256, 100, np.uint8)
    seeds = cf.seed_stream(60, start=3)
    mvp1, mvp2 = cf.default_mvp_inverse(), cf.golden_mvp("orbit")
    gpu.reset(mvp1, seeds[0])
    cpu.reset(mvp1, seeds[0], nthreads=16)
    k = 1
    for light, mvp, n in (((1, 0, 0), mvp1, 12), ((-1, 0, 0), mvp1, 12), ((-1, 0, 0), mvp2, 12),
                          ((0.6, 0.0, -0.8), mvp2, 12)):
        ld = np.asarray(light, np.float32)
        gpu.set_light(spd, ld)
        cpu.light, cpu.light_dir = spd, ld
        gpu.render_passes(mvp, seeds[k:k + n])
        for s in seeds[k:k + n]:
            rgb, want = cpu.render(mvp, s, nthreads=16)
        k += n
        what = f"dark, light {light}"
        assert_photons_equal(gpu.read_photons(), cpu.photons, what)
        assert_rgb32_equal(gpu.read_rgb(), rgb, what)
        assert_rgba_equal(gpu.read_rgba16f(), want, what)
    gpu.close()
