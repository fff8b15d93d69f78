"""Device-list handles (vptmcm_config::n_devices, SURVEY 8(b) "device list/mode"):
one handle drives N photon-parallel replicas, replica k on devices[k] with rank
k's seed stream, and the render target is their composite sum(rgb*n)/sum(n),
made on devices[0] by k_composite.

The box has one GPU, so the N > 1 cases repeat device 0 (VPTMCM_GROUP_PEER
allows it: the replicas then share the GPU and the peer copy is a device copy;
the code path is the one N GPUs take). Every result is checked bit for bit
against oracle replicas composited in the same order in numpy (f32 sums in
replica order, a correctly rounded f32 division, float16 round-to-nearest-even).
"""
import numpy as np
import pytest

import oracle as orc
import vptmcm
from vptmcm import configs as cf

from test_gpu_parity import assert_photons_equal, assert_rgb32_equal, assert_rgba_equal, make_pair

pytestmark = pytest.mark.gpu


def _setup(r, vol, tf, ext, spec="12"):
    spd, ld = np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32)
    r.set_spectrum(cf.spectrum_buffer(spec))
    r.set_volume(vol)
    r.set_material_tf(tf)
    r.set_light(spd, ld)
    r.set_params(extinction=ext, bounces=8, steps=8)


def _oracle_replica(R, vol, tf, ext, mvp, seeds):
    o = orc.Oracle(R)
    o.set_spectrum(cf.spectrum_buffer("12"))
    o.volume, o.tf, o.light, o.light_dir = vol, tf, np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32)
    o.params.update(extinction=ext, bounces=8, steps=8)
    o.reset(mvp, seeds[0], nthreads=16)
    rgb = None
    for s in seeds[1:]:
        rgb, _ = o.render(mvp, s, nthreads=16)
    return o, rgb


def _composite(replicas):
    """numpy restatement of k_composite over (oracle, rgb32) replicas."""
    tot = None
    for o, rgb in replicas:
        n = o.photons[:, 7].astype(np.float32).reshape(o.R, o.R)
        pack = np.concatenate([rgb * n[..., None], n[..., None]], axis=-1).astype(np.float32)
        tot = pack if tot is None else (tot + pack).astype(np.float32)
    n = tot[..., 3]
    with np.errstate(divide="ignore", invalid="ignore"):
        rgb = np.where(n[..., None] > 0, tot[..., :3] / n[..., None], np.float32(0)).astype(np.float32)
    half = rgb.astype(np.float16).view(np.uint16)
    rgba = np.concatenate([half, np.full(rgb.shape[:2] + (1,), 0x3C00, np.uint16)], axis=-1)
    return rgb, rgba, n


def test_group_of_one_is_the_single_device_renderer():
    """devices = [0]: the same photons and images as a plain device-0 handle and
    the oracle, bit for bit (no composite in the render target for N = 1); the
    explicit composite is (rgb*n)/n of that one replica."""
    R, vol, tf, mvp = 96, cf.fbm_volume(64, 31, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    seeds = cf.seed_stream(7, start=0)
    g = vptmcm.Renderer(R, devices=[0])
    _setup(g, vol, tf, 32.0)
    assert g.group_devices() == [0]
    gpu, _ = make_pair(R, vol, tf, ext=32.0)
    for r in (g, gpu):
        r.reset(mvp, seeds[0])
        r.render_passes(mvp, seeds[1:4])
        for s in seeds[4:]:
            r.render(mvp, s)
    o, rgb = _oracle_replica(R, vol, tf, 32.0, mvp, seeds)
    for what, r in (("group [0]", g), ("single", gpu)):
        assert_photons_equal(r.read_photons(), o.photons, what)
        assert_rgb32_equal(r.read_rgb(), rgb, what)
    assert np.array_equal(g.read_rgba16f(), gpu.read_rgba16f())
    want_rgb, want_rgba, want_n = _composite([(o, rgb)])
    q, crgb, n = g.read_composite_all()
    assert np.array_equal(n, want_n)
    assert_rgb32_equal(crgb, want_rgb, "composite of one")
    assert np.array_equal(q, want_rgba)
    g.close()
    gpu.close()


@pytest.mark.parametrize("n_rep,threads", [(2, "1"), (3, "1"), (3, "0"), (8, "1")])
def test_group_replicas_composite_bitexact(n_rep, threads, monkeypatch):
    """N replicas on one GPU (devices = [0] * N): replica k marches with rank
    k's seed stream (the stream bench.py gives rank k, configs.seed_bits), the
    render target, the fp32 image and the tone mapper see the composite, and
    every output is bit-exact against N oracle replicas composited in replica
    order. Replica 0's photons are the handle's photons. Forwarded operations
    run on the per-replica worker threads, or serially on the caller's thread
    with VPTMCM_GROUP_THREADS=0: the same bits."""
    monkeypatch.setenv("VPTMCM_GROUP_THREADS", threads)
    R, vol, tf, mvp = 96, cf.fbm_volume(64, 32, nthreads=8), cf.tf_spectral(), cf.golden_mvp("orbit")
    base = cf.seed_stream(6, start=0)
    g = vptmcm.Renderer(R, devices=[0] * n_rep)
    _setup(g, vol, tf, 24.0)
    assert g.group_devices() == [0] * n_rep
    g.reset(mvp, base[0])
    g.render_passes(mvp, base[1:3])
    for s in base[3:]:
        g.render(mvp, s)
    reps = [_oracle_replica(R, vol, tf, 24.0, mvp, cf.seed_stream(6, start=0, rank=k)) for k in range(n_rep)]
    assert_photons_equal(g.read_photons(), reps[0][0].photons, "replica 0")
    want_rgb, want_rgba, want_n = _composite(reps)
    assert_rgb32_equal(g.read_rgb(), want_rgb, f"{n_rep}-replica composite fp32")
    assert_rgba_equal(g.read_rgba16f(), want_rgba, f"{n_rep}-replica composite rgba16f")
    q, crgb, n = g.read_composite_all()
    assert np.array_equal(n, want_n) and np.array_equal(q, want_rgba)
    # one more pass after an explicit (asynchronous) composite: the target follows the frame
    g.composite()
    g.render(mvp, base[-1] ^ 0x5555)
    reps = [_oracle_replica(R, vol, tf, 24.0, mvp,
                            np.append(cf.seed_stream(6, start=0, rank=k),
                                      np.uint32(cf.pcg((int(base[-1]) ^ 0x5555) ^ ((k * 0x9E3779B9) & 0xFFFFFFFF))
                                                if k else int(base[-1]) ^ 0x5555)))
            for k in range(n_rep)]
    want_rgb, want_rgba, _ = _composite(reps)
    assert_rgba_equal(g.read_rgba16f(), want_rgba, "composite after one more pass")
    g.close()


def _oracle_replicas_stepwise(R, vol, tf, ext, mvp, n_rep, n_pass, start=0):
    """N oracle replicas advanced one pass at a time: the composite after each pass."""
    reps, out = [], []
    for k in range(n_rep):
        o = orc.Oracle(R)
        o.set_spectrum(cf.spectrum_buffer("12"))
        o.volume, o.tf, o.light, o.light_dir = vol, tf, np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32)
        o.params.update(extinction=ext, bounces=8, steps=8)
        reps.append([o, None, cf.seed_stream(n_pass + 1, start=start, rank=k)])
    for o, _, sd in reps:
        o.reset(mvp, sd[0], nthreads=16)
    for p in range(1, n_pass + 1):
        for r in reps:
            r[1], _ = r[0].render(mvp, r[2][p], nthreads=16)
        out.append(_composite([(r[0], r[1]) for r in reps]))
    return out


@pytest.mark.parametrize("R,n_rep", [(64, 3), (16, 3), (40, 8)])
def test_group_per_pass_composites_bitexact(R, n_rep):
    """A composite after every pass, issued asynchronously (composite() after
    each render(), nothing read in between), so consecutive composites
    alternate the double-buffered packs and overlap the next passes; reads at
    two points and at the end equal the oracle replicas' composite after that
    many passes. R = 16 with 3 replicas leaves two of the three pixel shards
    empty; R = 40 is not a multiple of the 256-pixel shard unit."""
    vol, tf, mvp = cf.fbm_volume(48, 35, nthreads=8), cf.tf_spectral(), cf.golden_mvp("orbit")
    n_pass = 7
    want = _oracle_replicas_stepwise(R, vol, tf, 24.0, mvp, n_rep, n_pass, start=9)
    base = cf.seed_stream(n_pass + 1, start=9)
    g = vptmcm.Renderer(R, devices=[0] * n_rep)
    _setup(g, vol, tf, 24.0)
    g.reset(mvp, base[0])
    for p in range(1, n_pass + 1):
        g.render(mvp, base[p])
        g.composite()
        if p in (2, 5):
            q, crgb, n = g.read_composite_all()
            assert_rgb32_equal(crgb, want[p - 1][0], f"composite after pass {p}")
            assert np.array_equal(q, want[p - 1][1]) and np.array_equal(n, want[p - 1][2])
    g.synchronize()
    assert_rgb32_equal(g.read_rgb(), want[-1][0], "final composite fp32")
    assert_rgba_equal(g.read_rgba16f(), want[-1][1], "final composite rgba16f")
    q, crgb, n = g.read_composite_all()
    assert np.array_equal(n, want[-1][2])
    g.close()


def test_group_tonemap_reads_the_composite():
    R, vol, tf, mvp = 64, cf.fbm_volume(48, 33, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    seeds = cf.seed_stream(4, start=0)
    g = vptmcm.Renderer(R, devices=[0, 0])
    _setup(g, vol, tf, 16.0)
    g.reset(mvp, seeds[0])
    g.render_passes(mvp, seeds[1:])
    ldr = g.tonemap_artistic(0.0, 0.5, 1.0, 1.0, 2.2)
    # the same tone mapping on a single handle whose render target is replaced
    # by the composite: compare through the rgba16f target both see
    single = vptmcm.Renderer(R, device=0)
    _setup(single, vol, tf, 16.0)
    single.reset(mvp, seeds[0])
    single.render_passes(mvp, seeds[1:])
    assert not np.array_equal(single.read_rgba16f(), g.read_rgba16f())
    assert ldr.shape == (R, R, 4) and (ldr[..., 3] == 255).all()
    g2 = vptmcm.Renderer(R, devices=[0, 0])
    _setup(g2, vol, tf, 16.0)
    g2.reset(mvp, seeds[0])
    g2.render_passes(mvp, seeds[1:])
    assert np.array_equal(g2.tonemap_artistic(0.0, 0.5, 1.0, 1.0, 2.2), ldr)
    for r in (g, g2, single):
        r.close()


def test_group_rccl_transport_one_device():
    """VPTMCM_GROUP_RCCL: ncclCommInitAll over the device list and a grouped
    ncclReduce to devices[0], then k_composite. On a one-GPU box the list can
    only be [0]; the composite is (rgb*n)/n of that replica, bit-exact, and the
    render target stays the replica's own image (N = 1)."""
    R, vol, tf, mvp = 64, cf.fbm_volume(48, 34, nthreads=8), cf.tf_spectral(), cf.default_mvp_inverse()
    seeds = cf.seed_stream(4, start=0)
    g = vptmcm.Renderer(R, devices=[0], transport=vptmcm.GROUP_RCCL)
    _setup(g, vol, tf, 16.0)
    g.reset(mvp, seeds[0])
    g.render_passes(mvp, seeds[1:])
    o, rgb = _oracle_replica(R, vol, tf, 16.0, mvp, seeds)
    want_rgb, want_rgba, want_n = _composite([(o, rgb)])
    q, crgb, n = g.read_composite_all()
    assert np.array_equal(n, want_n)
    assert_rgb32_equal(crgb, want_rgb, "RCCL composite")
    assert np.array_equal(q, want_rgba)
    assert_rgb32_equal(g.read_rgb(), rgb, "RCCL group render target")
    g.close()


def test_group_argument_errors():
    with pytest.raises(vptmcm.VptError, match="distinct devices") as e:
        vptmcm.Renderer(16, devices=[0, 0], transport=vptmcm.GROUP_RCCL)
    assert e.value.code == vptmcm.EINVAL
    with pytest.raises(vptmcm.VptError, match="not a device ordinal"):
        vptmcm.Renderer(16, devices=[0, 4096])
    with pytest.raises(vptmcm.VptError, match="transport"):
        vptmcm.Renderer(16, devices=[0], transport=7)
    g = vptmcm.Renderer(16, devices=[0, 0])
    with pytest.raises(vptmcm.VptError, match="composites its replicas itself") as e:
        g.comm_init(vptmcm.unique_id(), 1, 0)
    assert e.value.code == vptmcm.ESTATE
    with pytest.raises(vptmcm.VptError, match="no volume"):
        g.render(cf.default_mvp_inverse(), 1)
    g.close()


def test_group_rgb_sibling_composites():
    """The RGB sibling ('mcm-compute') behind a device list: two replicas on one
    GPU, composited like the spectral renderer's; its fp32 image is the photon's
    radiance (MCMComputeRenderer.wgsl:161), so the oracle composite is built
    from the oracle photons."""
    from test_gpu_rgb import tf_rgb
    R, vol, mvp = 64, cf.fbm_volume(48, 13, nthreads=8), cf.default_mvp_inverse()
    tf, env = tf_rgb("ramp"), (255, 230, 200, 255)
    g = vptmcm.Renderer(R, devices=[0, 0], renderer=vptmcm.RENDERER_RGB)
    g.set_transfer_function(tf)
    g.set_environment(env)
    g.set_volume(vol)
    g.set_params(extinction=24.0, anisotropy=0.6, bounces=8, steps=8)
    base = cf.seed_stream(6, start=40)
    g.reset(mvp, base[0])
    g.render_passes(mvp, base[1:])
    reps = []
    for k in (0, 1):
        o = orc.OracleRGB(R)
        o.volume, o.tf, o.env = vol, tf, np.array(env, np.uint8)
        o.params.update(extinction=24.0, anisotropy=0.6, bounces=8, steps=8)
        s = cf.seed_stream(6, start=40, rank=k)
        o.reset(mvp, s[0])
        for x in s[1:]:
            o.render(mvp, x)
        rgb = o.photons.reshape(R, R, -1)[..., 12:15].copy().view(np.float32)
        reps.append((o, rgb))
    assert (g.read_photons() == reps[0][0].photons).all()
    want_rgb, want_rgba, _ = _composite(reps)
    assert_rgb32_equal(g.read_rgb(), want_rgb, "RGB sibling composite")
    assert_rgba_equal(g.read_rgba16f(), want_rgba, "RGB sibling composite")
    g.close()


def test_bench_launcherless_two_gpus_repeated_device():
    """bench.py --gpus 2 without a launcher on the one-GPU box (VERDICT r04
    next 1): the test-only VPTMCM_BENCH_DEVICES=0,0 repeats device 0, so the
    launcher-less path runs end to end on hardware — one process, one
    2-replica device-list handle, each timed region ending with the PEER
    composite — and the line reports 2 GPUs, the device list and the
    transport. (Two replicas share one GPU here, so the value says nothing
    about N-GPU scaling: N > 1 distinct GPUs stay unmeasured.)"""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env["VPTMCM_BENCH_DEVICES"] = "0,0"
    p = subprocess.run([sys.executable, str(repo / "bench.py"), "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--volume", "64", "--resolution", "64", "--cpu-seconds", "0", "--settle-ms", "20",
                        "--per-pass-steps", "8"], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr[-3000:]
    rec = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_gpus"] == 2 and rec["config"]["devices"] == [0, 0]
    assert rec["config"]["composite_transport"] == "peer-sharded" and "one process" in rec["config"]["parallelism"]
    assert rec["value"] > 0 and rec["per_pass_allreduce"]["value"] > 0
    assert rec["roofline"]["passes_per_launch"] == 20
