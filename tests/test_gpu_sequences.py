"""Random operation sequences on one renderer against the oracle.

The other parity tests fix a short script per handle (reset, a few passes, a
read); the library, though, carries state from launch to launch: queued
render() passes fused into one launch at the next observation, the tile
schedule's flags and the deal kept while they do not change, the completion
signal, parameter and table changes flushing the queue first. Here each case
drives one handle through a seeded random sequence of 20-50 operations —
render, render_passes of 1-40 passes, camera switches between three matrices,
reset, extinction / bounces / steps / blur changes, a new TF, light or bin
layout, and reads — with the oracle mirroring every operation in the same
order; every read compares the photons (and, after a pass, both images) bit
for bit. VPTMCM_SEQ_CASES / VPTMCM_SEQ_BASE: a longer campaign over fresh
sequences (tools/fuzz_campaign.sh runs them with the random-configuration
tests)."""
import os

import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf
from test_gpu_fuzz import _perspective_inverse, _spectrum, _tf, _volume
from test_gpu_parity import assert_photons_equal, assert_rgb32_equal, assert_rgba_equal

pytestmark = pytest.mark.gpu

N_SEQ = int(os.environ.get("VPTMCM_SEQ_CASES", "8"))
BASE = int(os.environ.get("VPTMCM_SEQ_BASE", "0"))
_OPS = ["render", "passes", "camera", "reset", "params", "tf", "light", "spectrum", "read"]
_P = [0.22, 0.2, 0.12, 0.06, 0.1, 0.05, 0.05, 0.05, 0.15]


def _light(rng):
    iso = rng.random() < 0.2
    ld = np.zeros(3, np.float32) if iso else rng.normal(size=3).astype(np.float32)
    spd = (np.full(256, 100, np.uint8) if rng.random() < 0.5
           else rng.integers(0, 256, 256, dtype=np.uint8))
    return spd, ld


def _params(rng):
    ext = float(np.float32(10 ** rng.uniform(-0.3, 2.2)))
    ext = {0: 0.0}.get(int(rng.integers(0, 25)), ext)
    return dict(extinction=ext, bounces=int(rng.integers(0, 11)), steps=int(rng.integers(0, 17)),
                blur=float(np.float32(rng.uniform(0, 0.3))) if rng.random() < 0.15 else 0.0)


@pytest.mark.parametrize("k", range(N_SEQ))
def test_random_operation_sequence_bitexact(k):
    rng = np.random.default_rng(50000 + BASE + k)
    R = int(rng.choice([16, 24, 40, 64, 72, 96])) + (int(rng.integers(1, 8)) if rng.random() < 0.25 else 0)
    layout = int(rng.choice([vptmcm.LAYOUT_LINEAR, vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_BRICK8,
                             vptmcm.LAYOUT_COLUMN4]))
    shape = tuple(int(x) for x in rng.integers(8, 64, 3)) if rng.random() < 0.4 else (48, 48, 48)
    vol = _volume(shape, int(rng.integers(0, 1 << 16)))
    mvps = [cf.default_mvp_inverse()] + [_perspective_inverse(rng, inside=rng.random() < 0.2)
                                         for _ in range(2)]
    seeds = iter(cf.seed_stream(2000, start=5000 * (BASE + k)).tolist())
    log = [f"case {k}: R={R} layout={layout} vol={shape}"]
    with vptmcm.Renderer(R, device=0, layout=layout) as gpu:
        cpu = orc.Oracle(R)
        _, spec = _spectrum(rng)
        _, tf = _tf(rng)
        spd, ld = _light(rng)
        params = _params(rng)
        gpu.set_spectrum(spec)
        cpu.set_spectrum(spec)
        gpu.set_volume(vol)
        cpu.volume = vol
        gpu.set_material_tf(tf)
        cpu.tf = tf
        gpu.set_light(spd, ld)
        cpu.light, cpu.light_dir = spd, ld
        gpu.set_params(**params)
        cpu.params.update(**params)
        cam = 0
        s = next(seeds)
        gpu.reset(mvps[cam], s)
        cpu.reset(mvps[cam], s, nthreads=16)
        img = None  # the oracle's last pass images (None right after a reset)

        def check(what):
            where = " / ".join(log[-6:])
            assert_photons_equal(gpu.read_photons(), cpu.photons, f"{what}: {where}")
            if img is not None:
                assert_rgb32_equal(gpu.read_rgb(), img[0], f"{what}: {where}")
                assert_rgba_equal(gpu.read_rgba16f(), img[1], f"{what}: {where}")

        for step in range(int(rng.integers(20, 51))):
            op = _OPS[int(rng.choice(len(_OPS), p=_P))]
            if op == "render":
                s = next(seeds)
                gpu.render(mvps[cam], s)
                img = cpu.render(mvps[cam], s, nthreads=16)
                log.append(f"render cam {cam}")
            elif op == "passes":
                n = int(rng.integers(1, 41))
                ss = [next(seeds) for _ in range(n)]
                gpu.render_passes(mvps[cam], ss)
                for s in ss:
                    img = cpu.render(mvps[cam], s, nthreads=16)
                log.append(f"{n} passes cam {cam}")
            elif op == "camera":
                cam = int(rng.integers(0, 3))
                log.append(f"camera {cam}")
            elif op == "reset":
                s = next(seeds)
                gpu.reset(mvps[cam], s)
                cpu.reset(mvps[cam], s, nthreads=16)
                img = None
                log.append(f"reset cam {cam}")
            elif op == "params":
                params = _params(rng)
                gpu.set_params(**params)
                cpu.params.update(**params)
                log.append(f"params {params}")
            elif op == "tf":
                what, tf = _tf(rng)
                gpu.set_material_tf(tf)
                cpu.tf = tf
                log.append(f"tf {what}")
            elif op == "light":
                spd, ld = _light(rng)
                gpu.set_light(spd, ld)
                cpu.light, cpu.light_dir = spd, ld
                log.append("light")
            elif op == "spectrum":
                what, spec = _spectrum(rng)
                gpu.set_spectrum(spec)
                cpu.set_spectrum(spec)
                log.append(f"spectrum {what}")
            else:
                check(f"step {step}")
                log.append("read")
        check("end")


def _replica_seed(s: int, j: int) -> int:
    """vptmcm.cpp replica_seed: replica j's seed bits for replica 0's s."""
    return s if j == 0 else cf.pcg((s ^ ((j * 0x9E3779B9) & 0xFFFFFFFF)) & 0xFFFFFFFF)


@pytest.mark.parametrize("k", range(max(1, N_SEQ // 2)))
def test_random_group_sequence_bitexact(k):
    """The same random sequences through a device-list handle of 2-4 replicas
    on device 0 (worker threads forwarding every call, replica j on its own
    seed stream), with explicit composites among the operations: every read
    compares replica 0's photons and the composite's fp32 and rgba16float
    images and sample counts with oracle replicas composited in replica order."""
    from test_gpu_group import _composite
    rng = np.random.default_rng(70000 + BASE + k)
    n_rep = int(rng.integers(2, 5))
    R = int(rng.choice([16, 24, 40, 64])) + (int(rng.integers(1, 8)) if rng.random() < 0.25 else 0)
    layout = int(rng.choice([vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_COLUMN4, vptmcm.LAYOUT_BRICK8]))
    vol = _volume((48, 48, 48), int(rng.integers(0, 1 << 16)))
    mvps = [cf.default_mvp_inverse()] + [_perspective_inverse(rng) for _ in range(2)]
    seeds = iter(cf.seed_stream(2000, start=5000 * (BASE + k) + 17).tolist())
    log = [f"group case {k}: x{n_rep} R={R} layout={layout}"]
    with vptmcm.Renderer(R, devices=[0] * n_rep, layout=layout) as g:
        cpus = [orc.Oracle(R) for _ in range(n_rep)]
        _, spec = _spectrum(rng)
        _, tf = _tf(rng)
        spd, ld = _light(rng)
        params = _params(rng)
        g.set_spectrum(spec)
        g.set_volume(vol)
        g.set_material_tf(tf)
        g.set_light(spd, ld)
        g.set_params(**params)
        for c in cpus:
            c.set_spectrum(spec)
            c.volume, c.tf, c.light, c.light_dir = vol, tf, spd, ld
            c.params.update(**params)
        cam = 0

        def each(fn):
            return [fn(j, c) for j, c in enumerate(cpus)]

        s = next(seeds)
        g.reset(mvps[cam], s)
        each(lambda j, c: c.reset(mvps[cam], _replica_seed(s, j), nthreads=16))
        imgs = None

        def check(what):
            where = " / ".join(log[-6:])
            assert_photons_equal(g.read_photons(), cpus[0].photons, f"{what}: {where}")
            if imgs is not None:
                want_rgb, want_rgba, want_n = _composite([(c, im[0]) for c, im in zip(cpus, imgs)])
                q, rgb, n = g.read_composite_all()
                assert np.array_equal(n, want_n), f"{what} counts: {where}"
                assert_rgb32_equal(rgb, want_rgb, f"{what}: {where}")
                assert_rgba_equal(q, want_rgba, f"{what}: {where}")

        for step in range(int(rng.integers(15, 36))):
            op = _OPS[int(rng.choice(len(_OPS), p=_P))]
            if op == "render":
                s = next(seeds)
                g.render(mvps[cam], s)
                imgs = each(lambda j, c: c.render(mvps[cam], _replica_seed(s, j), nthreads=16))
                log.append(f"render cam {cam}")
            elif op == "passes":
                ss = [next(seeds) for _ in range(int(rng.integers(1, 41)))]
                g.render_passes(mvps[cam], ss)
                for s in ss:
                    imgs = each(lambda j, c: c.render(mvps[cam], _replica_seed(s, j), nthreads=16))
                if rng.random() < 0.3:
                    g.composite()  # asynchronous, right after the frame
                log.append(f"{len(ss)} passes cam {cam}")
            elif op == "camera":
                cam = int(rng.integers(0, 3))
                log.append(f"camera {cam}")
            elif op == "reset":
                s = next(seeds)
                g.reset(mvps[cam], s)
                each(lambda j, c: c.reset(mvps[cam], _replica_seed(s, j), nthreads=16))
                imgs = None
                log.append(f"reset cam {cam}")
            elif op == "params":
                params = _params(rng)
                g.set_params(**params)
                each(lambda j, c: c.params.update(**params))
                log.append(f"params {params}")
            elif op == "tf":
                what, tf = _tf(rng)
                g.set_material_tf(tf)
                for c in cpus:
                    c.tf = tf
                log.append(f"tf {what}")
            elif op == "light":
                spd, ld = _light(rng)
                g.set_light(spd, ld)
                for c in cpus:
                    c.light, c.light_dir = spd, ld
                log.append("light")
            elif op == "spectrum":
                what, spec = _spectrum(rng)
                g.set_spectrum(spec)
                for c in cpus:
                    c.set_spectrum(spec)
                log.append(f"spectrum {what}")
            else:
                check(f"step {step}")
                log.append("read")
        check("end")


@pytest.mark.parametrize("k", range(max(1, N_SEQ // 2)))
def test_random_rgb_sequence_bitexact(k):
    """The RGB sibling ('mcm-compute') through random sequences: render,
    render_passes, camera switches, reset, extinction / anisotropy / bounces /
    steps changes, a new rgba8 TF image or environment colour, reads (photon
    words and the rgba16float image bit for bit, NaN == NaN)."""
    from test_gpu_fuzz import _same_words
    rng = np.random.default_rng(90000 + BASE + k)
    R = int(rng.choice([16, 24, 40, 64])) + (int(rng.integers(1, 8)) if rng.random() < 0.25 else 0)
    layout = int(rng.choice([vptmcm.LAYOUT_LINEAR, vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_BRICK8,
                             vptmcm.LAYOUT_COLUMN4]))
    vol = _volume((48, 48, 48), int(rng.integers(0, 1 << 16)))
    mvps = [cf.default_mvp_inverse()] + [_perspective_inverse(rng) for _ in range(2)]
    seeds = iter(cf.seed_stream(2000, start=5000 * (BASE + k) + 29).tolist())
    log = [f"rgb case {k}: R={R} layout={layout}"]

    def tf_img():
        return rng.integers(0, 256, (int(rng.integers(1, 4)), int(rng.integers(2, 300)), 4), dtype=np.uint8)

    def rgb_params():
        p = _params(rng)
        return dict(extinction=p["extinction"], anisotropy=float(np.float32(rng.uniform(-0.95, 0.95))),
                    bounces=p["bounces"], steps=p["steps"])

    with vptmcm.Renderer(R, device=0, layout=layout, renderer=vptmcm.RENDERER_RGB) as gpu:
        cpu = orc.OracleRGB(R)
        tf, env, params = tf_img(), tuple(int(x) for x in rng.integers(0, 256, 4)), rgb_params()
        gpu.set_transfer_function(tf)
        gpu.set_environment(env)
        gpu.set_volume(vol)
        gpu.set_params(**params)
        cpu.volume, cpu.tf, cpu.env = vol, tf, np.array(env, np.uint8)
        cpu.params.update(**params)
        cam = 0
        s = next(seeds)
        gpu.reset(mvps[cam], s)
        cpu.reset(mvps[cam], s)
        want = None

        def check(what):
            where = " / ".join(log[-6:])
            ok = _same_words(gpu.read_photons(), cpu.photons)
            assert ok.all(), f"{what}: {int((~ok).sum())} photon words differ: {where}"
            if want is not None:
                assert np.array_equal(gpu.read_rgba16f(), want), f"{what}: image differs: {where}"

        ops = ["render", "passes", "camera", "reset", "params", "tf", "env", "read"]
        probs = [0.24, 0.22, 0.12, 0.06, 0.1, 0.05, 0.05, 0.16]
        for step in range(int(rng.integers(15, 41))):
            op = ops[int(rng.choice(len(ops), p=probs))]
            if op == "render":
                s = next(seeds)
                gpu.render(mvps[cam], s)
                _, want = cpu.render(mvps[cam], s)
                log.append(f"render cam {cam}")
            elif op == "passes":
                ss = [next(seeds) for _ in range(int(rng.integers(1, 41)))]
                gpu.render_passes(mvps[cam], ss)
                for s in ss:
                    _, want = cpu.render(mvps[cam], s)
                log.append(f"{len(ss)} passes cam {cam}")
            elif op == "camera":
                cam = int(rng.integers(0, 3))
                log.append(f"camera {cam}")
            elif op == "reset":
                s = next(seeds)
                gpu.reset(mvps[cam], s)
                cpu.reset(mvps[cam], s)
                want = None
                log.append(f"reset cam {cam}")
            elif op == "params":
                params = rgb_params()
                gpu.set_params(**params)
                cpu.params.update(**params)
                log.append(f"params {params}")
            elif op == "tf":
                tf = tf_img()
                gpu.set_transfer_function(tf)
                cpu.tf = tf
                log.append(f"tf {tf.shape}")
            elif op == "env":
                env = tuple(int(x) for x in rng.integers(0, 256, 4))
                gpu.set_environment(env)
                cpu.env = np.array(env, np.uint8)
                log.append(f"env {env}")
            else:
                check(f"step {step}")
                log.append("read")
        check("end")


@pytest.mark.parametrize("k", range(max(1, N_SEQ // 2)))
def test_random_band_sequence_bitexact(k):
    """Mode B bands changing mid-sequence (vptmcm_set_band: reset and render
    touch only the band's rows, every other photon is left as it was): random
    sequences of render, render_passes, camera switches, reset, band changes
    (whole 8-row tiles, the last band ending at R) and parameter changes; every
    read compares the whole photon buffer and the rows the last pass rendered
    with the oracle's row-restricted run."""
    rng = np.random.default_rng(110000 + BASE + k)
    R = int(rng.choice([24, 40, 64, 72])) + (int(rng.integers(1, 8)) if rng.random() < 0.3 else 0)
    layout = int(rng.choice([vptmcm.LAYOUT_CORNER8, vptmcm.LAYOUT_COLUMN4, vptmcm.LAYOUT_BRICK8]))
    vol = _volume((48, 48, 48), int(rng.integers(0, 1 << 16)))
    mvps = [cf.default_mvp_inverse()] + [_perspective_inverse(rng) for _ in range(2)]
    seeds = iter(cf.seed_stream(2000, start=5000 * (BASE + k) + 41).tolist())
    tiles = (R + 7) // 8
    log = [f"band case {k}: R={R} layout={layout}"]

    def new_band():
        if rng.random() < 0.2:
            return 0, R
        a = int(rng.integers(0, tiles))
        b = int(rng.integers(a + 1, tiles + 1))
        return 8 * a, min(R, 8 * b)

    with vptmcm.Renderer(R, device=0, layout=layout) as gpu:
        cpu = orc.Oracle(R)
        _, spec = _spectrum(rng)
        _, tf = _tf(rng)
        spd, ld = _light(rng)
        params = _params(rng)
        gpu.set_spectrum(spec)
        cpu.set_spectrum(spec)
        gpu.set_volume(vol)
        cpu.volume = vol
        gpu.set_material_tf(tf)
        cpu.tf = tf
        gpu.set_light(spd, ld)
        cpu.light, cpu.light_dir = spd, ld
        gpu.set_params(**params)
        cpu.params.update(**params)
        band = (0, R)
        cam = 0

        def reset_both(s):
            gpu.reset(mvps[cam], s)
            keep = cpu.photons.copy()
            cpu.reset(mvps[cam], s, nthreads=16)
            rows = np.zeros((R, R), bool)
            rows[band[0]:band[1]] = True
            cpu.photons[~rows.reshape(-1)] = keep[~rows.reshape(-1)]

        reset_both(next(seeds))
        img = None
        # per image row: 1 = the last pass's row (compare with img), 2 = zero
        # (fp32 rows outside a band set since), 0 = not modelled (an older pass)
        fp_rows = np.zeros(R, np.int8)
        q_rows = np.zeros(R, bool)  # rgba16f rows of the last pass (band changes leave them)

        def check(what):
            where = " / ".join(log[-6:])
            assert_photons_equal(gpu.read_photons(), cpu.photons, f"{what}: {where}")
            got = gpu.read_rgb()
            assert not got[fp_rows == 2].any(), f"{what}: fp32 rows zeroed by a band change: {where}"
            if img is not None:
                assert_rgb32_equal(got[fp_rows == 1], img[0][fp_rows == 1], f"{what}: {where}")
                assert_rgba_equal(gpu.read_rgba16f()[q_rows], img[1][q_rows], f"{what}: {where}")

        ops = ["render", "passes", "camera", "reset", "band", "params", "read"]
        probs = [0.22, 0.2, 0.1, 0.1, 0.13, 0.08, 0.17]
        for step in range(int(rng.integers(15, 41))):
            op = ops[int(rng.choice(len(ops), p=probs))]
            if op in ("render", "passes"):
                ss = ([next(seeds)] if op == "render"
                      else [next(seeds) for _ in range(int(rng.integers(1, 41)))])
                if op == "render":
                    gpu.render(mvps[cam], ss[0])
                else:
                    gpu.render_passes(mvps[cam], ss)
                for s in ss:
                    img = cpu.render(mvps[cam], s, nthreads=16, rows=band)
                fp_rows[fp_rows == 1] = 0
                fp_rows[band[0]:band[1]] = 1
                q_rows[:] = False
                q_rows[band[0]:band[1]] = True
                log.append(f"{len(ss)} pass(es) cam {cam} band {band}")
            elif op == "camera":
                cam = int(rng.integers(0, 3))
                log.append(f"camera {cam}")
            elif op == "reset":
                reset_both(next(seeds))
                img = None
                log.append(f"reset cam {cam} band {band}")
            elif op == "band":
                band = new_band()
                gpu.set_band(*band)
                fp_rows[:band[0]] = 2
                fp_rows[band[1]:] = 2
                log.append(f"band {band}")
            elif op == "params":
                params = _params(rng)
                gpu.set_params(**params)
                cpu.params.update(**params)
                log.append(f"params {params}")
            else:
                check(f"step {step}")
                log.append("read")
        check("end")
