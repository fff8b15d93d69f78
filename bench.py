#!/usr/bin/env python3
"""Benchmark of the spectral MCM photon march (BASELINE.json metric).

One "step" = one progressive pass of the hot path: R^2 photons x S photon-steps
(MCMSpectralComputeRenderer.wgsl:123-164), plus — at N > 1 — the RCCL all-reduce
of the (rgb*n, n) radiance buffer that composites the photon-parallel replicas.

Workload (BASELINE.md C3 at N = 1, C4 at N = 8): 512^3 fBm volume (seed 512),
spectral TF with HG g = 0.702, R = 512, S = 8, 12 bins, extinction 32, default
camera. Inputs are resident in HBM before the timed region.

Launch: `python bench.py --gpus N --steps K --warmup W`, or under
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`:
one process per GPU (LOCAL_RANK), RCCL bootstrapped torch-free (rendezvous.py).
Without a launcher (no WORLD_SIZE) and N > 1, one process drives the N GPUs
through one device-list handle (the north_star's one-process JS host shape:
replica k on device k, each compositing its 1/N pixel shard); it fails if fewer than N
devices are visible. Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
PKG = REPO / "vpt-spectral-volume-rendering_amd"
sys.path[:0] = [str(PKG / "python")]

import numpy as np  # noqa: E402

import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402
from vptmcm import rendezvous  # noqa: E402

METRIC = "Mphoton-steps/sec (+ achieved HBM GB/s), 512³ spectral MCM, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# 1024 SIMD-32 units x 2.4 GHz / 2 cycles per wave64 VALU instruction
VALU_PEAK_G = 1024 * 2.4 / 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1024, help="timed passes")
    # the engine clock ramps up over the first ~30 ms of sustained work (DVFS):
    # 4096 untimed passes (~65 ms) settle it, so the timed region measures the
    # sustained rate (measured: 19.8 us/pass after 0 warm-up passes, 18.2 after
    # 32, 17.4 after 512, 15.6-15.8 after 2048 and 8192)
    ap.add_argument("--warmup", type=int, default=4096, help="untimed passes")
    # The driver runs `--warmup 5`: 5 passes (~0.1 ms) leave the clock cold, so
    # a short timed region measured 18.7 us/pass against 15.7 sustained. Before
    # the W warm-up passes, untimed passes therefore run until this much wall
    # time has passed (reported as config.clock_settle_ms; 0 = off).
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed clock-settling passes before the warm-up (wall ms)")
    ap.add_argument("--resolution", type=int, default=512)
    ap.add_argument("--volume", type=int, default=512)
    ap.add_argument("--volume-kind", choices=["fbm", "two_spheres"], default="fbm",
                    help="fbm: the benchmark's fBm cloud (fills the cube); two_spheres: the "
                         "reference's test volume (generate_test_volume.ipynb) at that size, two "
                         "spheres in empty space (analysis only: empty-space traversal)")
    ap.add_argument("--photon-steps", type=int, default=8, help="S: steps per pass")
    ap.add_argument("--extinction", type=float, default=32.0)
    ap.add_argument("--layout", choices=["corner8", "brick8", "column4", "linear"], default="column4")
    ap.add_argument("--tf", choices=["spectral", "grey", "zero", "materials", "materials_const"],
                    default="spectral", help="TF (non-spectral: analysis only)")
    ap.add_argument("--bins", default="12", help="spectrum bin layout (non-12: analysis only)")
    ap.add_argument("--camera", choices=["default", "near", "orbit", "orbit_tilted"],
                    default="default", help="golden camera pose (non-default: analysis only)")
    ap.add_argument("--camera-mix", type=float, default=None,
                    help="analysis: blend the default and near cameras' inverse matrices, "
                         "(1 - t) * default + t * near, for intermediate screen coverage")
    ap.add_argument("--fuse", type=int, default=32,
                    help="passes per march launch (render_passes; photon state stays in "
                         "registers between them, every pass stores its image); 1 = one launch "
                         "per render() call")
    ap.add_argument("--allreduce-every", type=int, default=32,
                    help="passes between radiance composites (N > 1)")
    ap.add_argument("--transport", choices=["peer", "rccl"], default="peer",
                    help="N > 1 without a launcher: the device-list composite's transport "
                         "(peer: sharded, every GPU composites 1/N of the frame from every GPU's "
                         "(rgb*n, n) buffer over xGMI peer reads; rccl: ncclCommInitAll + grouped "
                         "ncclReduce to device 0)")
    ap.add_argument("--final-composite", choices=["inline", "side"], default="inline",
                    help="N > 1 under a launcher: the all-reduce that ends a region runs on the march "
                         "stream (inline: VPTMCM_ALLREDUCE_INLINE, no event hop to the side stream; "
                         "the composite is about to be read) or on the side stream like the ones "
                         "between launches, which overlap the next march")
    ap.add_argument("--shard-composite", choices=["on", "off"], default="on",
                    help="N > 1 under a launcher: the composites reduce-scatter (on: "
                         "VPTMCM_ALLREDUCE_SHARDED, each rank keeps the summed (rgb*n, n) of 1/N of the "
                         "pixels, half the all-reduce's traffic; reading the image all-gathers the shards, "
                         "as the device-list composite's readers do) or all-reduce (off)")
    ap.add_argument("--per-pass-steps", type=int, default=64,
                    help="N > 1: passes of a second timed region compositing after EVERY pass "
                         "(north_star's 'all-reduce each progressive pass'; one launch per pass; "
                         "reported as 'per_pass_allreduce'; 0 = skip)")
    ap.add_argument("--unfused-steps", type=int, default=64,
                    help="passes of a second timed region at one launch per pass (reported "
                         "as 'unfused'; 0 = skip; N = 1 only)")
    ap.add_argument("--api-steps", type=int, default=256,
                    help="passes of a third timed region through the drop-in render() entry "
                         "point, one call per pass (lazily fused by the library; reported as "
                         "'render_api'; 0 = skip; N = 1 only)")
    ap.add_argument("--js-steps", type=int, default=256,
                    help="passes of a timed region driven from Node through the drop-in JS "
                         "renderer (MCMSpectralComputeRenderer.render() per pass over N-API; "
                         "reported as 'js_api'; 0 = skip; N = 1 only)")
    ap.add_argument("--no-timing", action="store_true",
                    help="diagnostics: no per-launch kernel timestamps (wall clock only; the "
                         "roofline fields are then null)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="budget of the CPU-oracle baseline (0 = skip)")
    ap.add_argument("--rgb-steps", type=int, default=256,
                    help="passes of a timed region on the RGB sibling renderer ('mcm-compute', "
                         "MCMComputeRenderer.wgsl) on the same volume (reported as 'rgb'; "
                         "0 = skip; N = 1 only)")
    ap.add_argument("--general-steps", type=int, default=64,
                    help="passes of a timed region on the general (non-FAST) march: a UI-like "
                         "TF with wavelength-varying anisotropy and 8 uneven bins (reported as "
                         "'general'; 0 = skip; N = 1 only)")
    ap.add_argument("--near-steps", type=int, default=256,
                    help="passes of an analysis region with the golden 'near' camera (the volume fills "
                         "the frame: every photon-step is an in-volume gather), reported as 'near' with a "
                         "roofline of its own; 0 = skip; N = 1, default camera only")
    ap.add_argument("--traffic-json", default=str(REPO / "profiles" / "pmc_traffic.json"),
                    help="PMC-derived HBM bytes per launch (profiles/), if present")
    return ap.parse_args()


def cpu_baseline(vol, tf, spec, spd, ldir, mvp, R, S, ext, budget_s):
    """The north_star's CPU baseline: the scalar JavaScript re-execution of the
    same march (oracle/mcm_march.js, bit-exact with the C oracle) under
    worker_threads on this host's cores, full R^2 frames until the budget is
    spent. The C oracle on the same threads is reported beside it ('c_port')."""
    sys.path.insert(0, str(REPO / "oracle"))
    import js_march  # test-infrastructure restatement, timed here as the CPU baseline
    import oracle as orc  # test-infrastructure checker, timed as the secondary baseline

    # threads = the CPUs in this process's affinity mask, capped by the cgroup's
    # CPU quota and by OMP_NUM_THREADS when set; the machine may report many more
    threads = cf.host_threads()
    hs = cf.host_cpu_share()
    q = hs["cgroup_quota_cpus"]
    share = (f"{threads} threads = min(affinity mask {hs['affinity']} CPUs, cgroup cpu quota "
             f"{'unlimited' if q is None else f'{q:g} CPUs'}, OMP_NUM_THREADS="
             f"{hs['omp_num_threads'] or 'unset'}); os.cpu_count() {hs['os_cpu_count']}")
    out = None
    if js_march.node():
        j = js_march.run_bench(R, vol, tf, spd, ldir, spec, mvp, cf.seed_stream(64, start=0),
                               threads, budget_s, extinction=ext, bounces=8, steps=S)
        out = {"value": round(j["photon_steps_per_s"] / 1e6, 3), "unit": "Mphoton-steps/s",
               "cores": threads, "kind": "port", "host_cpus": os.cpu_count(),
               "sample": f"JavaScript re-execution (oracle/mcm_march.js, Math.fround, node "
                         f"{j['node']} worker_threads x{j['threads']}), {j['passes']} full passes "
                         f"of the same {R}x{R}x{S} workload after 1 warm-up pass, "
                         f"{j['seconds']:.1f} s, {share}"}

    o = orc.Oracle(R)
    o.set_spectrum(spec)
    o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ldir
    o.params.update(extinction=ext, bounces=8, steps=S)
    o.reset(mvp, cf.seed_bits(0), nthreads=threads)
    o.render(mvp, cf.seed_bits(1), nthreads=threads)  # warm-up pass
    passes, t0 = 0, time.perf_counter()
    while True:
        o.render(mvp, cf.seed_bits(2 + passes), nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    c_port = {"value": round(R * R * S * passes / el / 1e6, 3), "unit": "Mphoton-steps/s",
              "cores": threads, "kind": "port",
              "sample": f"C oracle (oracle/mcm_oracle.c), {passes} full passes after 1 warm-up "
                        f"pass, {el:.1f} s, {threads} pthreads"}
    if out is None:  # no node on this host: the C port is the baseline
        out = dict(c_port, host_cpus=os.cpu_count())
    else:
        out["c_port"] = c_port
    return out


def js_api_line(vol, tf, spec, R, S, ext, passes, settle_ms):
    """The north_star host: Node drives MCMSpectralComputeRenderer (js/) with one
    render() per pass, as the reference's rendering loop does, over the N-API
    shim into the same library (tools/js_render_bench.js). Runs in its own
    process on the same GPU after this process's regions have drained."""
    import shutil
    import subprocess
    import tempfile
    if shutil.which("node") is None:
        return None
    with tempfile.TemporaryDirectory(prefix="vptmcm-js-") as d:
        d = Path(d)
        np.ascontiguousarray(vol).tofile(d / "vol.raw")
        np.ascontiguousarray(tf, np.uint8).tofile(d / "tf.bin")
        np.ascontiguousarray(spec, np.float32).tofile(d / "spec.bin")
        D, H, W = vol.shape
        case = dict(R=R, W=W, H=H, D=D, volume_path=str(d / "vol.raw"), tf_path=str(d / "tf.bin"),
                    spectrum_path=str(d / "spec.bin"), extinction=ext, steps=S,
                    settle_ms=settle_ms, warmup=64, passes=passes)
        (d / "case.json").write_text(json.dumps(case))
        p = subprocess.run(["node", str(REPO / "tools" / "js_render_bench.js"), str(d / "case.json")],
                           capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise RuntimeError(f"js_render_bench.js failed ({p.returncode}): {p.stderr[-2000:]}")
    j = json.loads(p.stdout.strip().splitlines()[-1])
    return {"value": round(j["value"], 3), "ms_per_step": round(j["ms_per_step"], 5),
            "steps": j["steps"], "launches": j["launches"],
            "note": f"node {j['node']}: MCMSpectralComputeRenderer.render() once per pass (each "
                    "re-sending the unchanged uniforms, as the reference does) over N-API; the "
                    "library fuses the queued passes into 32-pass launches"}


def stdout_to_stderr(fn):
    """Run fn with the process's stdout (fd 1) pointed at stderr: RCCL prints
    a version banner on stdout when a process creates its first communicator,
    and rank 0's stdout must carry the JSON line only."""
    import ctypes
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        return fn()
    finally:
        ctypes.CDLL(None).fflush(None)  # C stdio buffers, before fd 1 is restored
        os.dup2(saved, 1)
        os.close(saved)


def pmc_entry(a, R: int, S: int, shapes: list, camera: str, macro: bool = False):
    """The PMC passes' entry (profiles/pmc_traffic.json, tools/pmc_report.py) of
    exactly this launch shape — R, S, layout, volume, passes per launch,
    camera, macro-cell bound on or off — with the benchmark TF and bins, or None."""
    tp = Path(a.traffic_json)
    if not tp.exists() or len(shapes) != 1 or a.tf != "spectral" or a.bins != "12":
        return None
    try:
        t = json.loads(tp.read_text())
    except (ValueError, OSError):
        return None
    for e in t.get("entries", [t]):
        if (e.get("resolution") == R and e.get("steps") == S and e.get("layout") == a.layout
                and e.get("volume", 512) == a.volume and e.get("passes_per_launch", 1) == shapes[0]
                and e.get("camera", "default") == camera and e.get("macro_skip", False) == macro):
            e = dict(e)
            e["_source"] = f"{tp.relative_to(REPO) if tp.is_relative_to(REPO) else tp}"
            e["_gather_peak"] = t.get("gather_peak")
            return e
    return None


def group_devices(n: int) -> list:
    """The device list of the launcher-less N-GPU run: 0..N-1, or the
    comma-separated VPTMCM_BENCH_DEVICES (test-only override, e.g. "0,0" to
    run the control flow with a repeated device on a one-GPU box)."""
    v = os.environ.get("VPTMCM_BENCH_DEVICES")
    devs = [int(x) for x in v.split(",")] if v else list(range(n))
    if len(devs) != n:
        raise SystemExit(f"VPTMCM_BENCH_DEVICES={v!r} names {len(devs)} devices, --gpus {n}")
    return devs


TF_DESC = {"spectral": "spectral TF (HG g=0.702)", "grey": "grey TF", "zero": "zero TF",
           "materials": "UI-like materials TF (varying anisotropy)",
           "materials_const": "UI-like materials TF (constant anisotropy)"}


def volume_seed(n: int) -> int:
    """BASELINE.md's fBm seeds: C3's 512^3 volume seed 512, C5's 1024^3 seed 1024."""
    return 512 if n == 512 else n


def config_name(volume: int, n_gpus: int) -> str:
    """The BASELINE.json config a line measures (C3 / C4: 512^3 on 1 / N GPUs; C5: 1024^3)."""
    if volume == 512:
        return "C4" if n_gpus > 1 else "C3"
    if volume == 1024:
        return "C5" if n_gpus > 1 else "C5 (one GPU)"
    return "custom"


def main():
    a = parse()
    rank, world, local = rendezvous.env_world()
    group = 1  # GPUs this process drives (a device-list handle when > 1)
    if world != a.gpus:
        if "WORLD_SIZE" in os.environ:
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
        world, group = 1, a.gpus
    if rank != 0:
        # only rank 0's stdout carries the JSON line: everything the other
        # ranks' libraries print (RCCL's banner, warnings) goes to stderr
        sys.stdout.flush()
        os.dup2(2, 1)
    R, S = a.resolution, a.photon_steps
    layout = {"corner8": vptmcm.LAYOUT_CORNER8, "brick8": vptmcm.LAYOUT_BRICK8,
              "column4": vptmcm.LAYOUT_COLUMN4, "linear": vptmcm.LAYOUT_LINEAR}[a.layout]

    # ---- inputs (synthetic)
    t = time.perf_counter()
    vol = (cf.fbm_volume(a.volume, volume_seed(a.volume)) if a.volume_kind == "fbm"
           else cf.two_spheres(a.volume))
    gen_s = time.perf_counter() - t
    tf = {"spectral": cf.tf_spectral, "grey": cf.tf_grey, "zero": cf.tf_zero,
          "materials": lambda: cf.tf_materials(True),
          "materials_const": lambda: cf.tf_materials(False)}[a.tf]()
    spd, ldir = cf.light_default()
    spec = cf.spectrum_buffer(a.bins)
    mvp = cf.default_mvp_inverse() if a.camera == "default" else cf.golden_mvp(a.camera)
    if a.camera_mix is not None:
        t = np.float64(a.camera_mix)
        mvp = ((1 - t) * cf.default_mvp_inverse().astype(np.float64)
               + t * cf.golden_mvp("near").astype(np.float64)).astype(np.float32)

    # VPTMCM_BENCH_DEVICE pins every rank to one ordinal (rehearsing the N > 1
    # path on a one-GPU box); the default is one GPU per local rank
    device = int(os.environ.get("VPTMCM_BENCH_DEVICE", local))
    grouped = group > 1
    devs = group_devices(group) if grouped else [device]
    transport = {"peer": vptmcm.GROUP_PEER, "rccl": vptmcm.GROUP_RCCL}[a.transport]
    if grouped:
        try:
            r = vptmcm.Renderer(R, layout=layout, devices=devs, transport=transport)
        except vptmcm.VptError as e:  # e.g. fewer than N devices visible
            raise SystemExit(f"--gpus {group} without a launcher drives devices {devs} from one "
                             f"process through one device-list handle, and that failed: {e}")
    else:
        r = vptmcm.Renderer(R, device=device, layout=layout)
    r.set_volume(vol)
    r.set_material_tf(tf)
    r.set_light(spd, ldir)
    r.set_spectrum(spec)
    r.set_params(extinction=a.extinction, bounces=8, steps=S)

    # VPTMCM_BENCH_FORCE_COMM=1: the N > 1 code path (RCCL communicator,
    # composites, barriers, max-over-ranks) with however many ranks there are,
    # e.g. one: a hardware check of that path on a one-GPU box
    multi = world > 1 or (os.environ.get("VPTMCM_BENCH_FORCE_COMM") == "1" and not grouped)
    if multi:
        key = rendezvous.job_key()
        # every peer alive before any rank enters RCCL's bootstrap (bounded;
        # a missing rank ends the job here with ECOMM)
        rendezvous.join(rank, world, key=key)
        uid = stdout_to_stderr(lambda: rendezvous.exchange_unique_id(rank, vptmcm.unique_id, key=key))
        # RCCL's init cannot be bounded from inside the process (it does not
        # return while a peer that joined and then died is missing): a
        # watchdog ends the process instead, so the launcher tears the job down
        import threading

        def _init_hung():
            sys.stderr.write(f"rank {rank}: RCCL communicator init did not return within "
                             f"{rendezvous.default_timeout_s():g} s (a peer died after the rendezvous?)\n")
            sys.stderr.flush()
            os._exit(3)
        dog = threading.Timer(rendezvous.default_timeout_s(), _init_hung)
        dog.daemon = True
        dog.start()
        stdout_to_stderr(lambda: r.comm_init(uid, world, rank))
        dog.cancel()
        r.barrier()
        if rank == 0:
            rendezvous.cleanup(key, world)

    # the composite that ends a region (and runs every `every` passes): the
    # RCCL all-reduce across ranks, or the device-list handle's composite
    shard = a.shard_composite == "on"
    composite = ((lambda: r.allreduce_radiance(sharded=shard)) if multi
                 else (r.composite if grouped else None))
    # the composite that ends a region (what the display reads next)
    composite_last = composite
    if multi and a.final_composite == "inline":
        composite_last = lambda: r.allreduce_radiance(inline=True, sharded=shard)  # noqa: E731
    single = not multi and not grouped
    n_unfused = a.unfused_steps if single else 0
    n_api = a.api_steps if single else 0
    n_pp = a.per_pass_steps if not single else 0
    n_uwarm = 32 if n_unfused > 0 else 0  # untimed one-pass launches ahead of the unfused region
    seeds = cf.seed_stream(a.warmup + a.steps + n_unfused + n_api + n_pp + n_uwarm + 1, start=0, rank=rank)
    F = max(1, min(a.fuse, 32))
    every = max(1, a.allreduce_every)

    def passes_on(sd, first: int, count: int, F: int = F, m=mvp) -> list:
        launches, done = [], 0
        while done < count:
            n = min(F, count - done)
            r.render_passes(m, sd[first + done:first + done + n])
            launches.append(n)
            done += n
        return launches

    def passes(first: int, count: int, F: int = F, every: int = every) -> list:
        """Enqueue `count` passes from seeds[first:] in launches of <= F passes,
        compositing across ranks whenever `every` passes have completed and
        after the region's last pass (so every region ends with a composite
        the display could show). Returns the pass count of every march launch."""
        launches, done = [], 0
        if composite is None and F == 32:
            # one call: the library launches it in 32-pass launches
            r.render_passes(mvp, seeds[first:first + count])
            return [min(32, count - k) for k in range(0, count, 32)]
        while done < count:
            n = min(F, count - done)
            if composite:  # never fuse across a composite
                n = min(n, every - (first - 1 + done) % every)
            r.render_passes(mvp, seeds[first + done:first + done + n])
            launches.append(n)
            done += n
            if composite and ((first - 1 + done) % every == 0 or done == count):
                (composite_last if done == count else composite)()
        return launches

    r.reset(mvp, seeds[0])
    # no garbage-collector pause inside a timed region (a ~330 us driver region
    # is short enough for one to show): collect now, then keep it off
    gc.collect()
    gc.disable()
    # clock settling: launches of F passes (seeds from a stream of their own)
    # until settle_ms of wall time have passed, then the W warm-up passes
    settle_passes, t_settle = 0, time.perf_counter()
    if a.settle_ms > 0:
        sseeds = cf.seed_stream(F, start=1 << 20, rank=rank)
        while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
            for _ in range(8):
                r.render_passes(mvp, sseeds)
                settle_passes += F
            r.synchronize()
    settle_ms = (time.perf_counter() - t_settle) * 1e3
    passes(1, a.warmup)
    r.synchronize()
    if multi:
        r.barrier()

    # ---- timed region: K passes (+ composites), bracketed by barrier + sync
    r.enable_kernel_timing(not a.no_timing)
    stamps = os.environ.get("VPTMCM_BENCH_STAMPS")  # host clocks of the region (tools/wall_split.py)
    if stamps:
        clk = [(time.clock_gettime_ns(time.CLOCK_MONOTONIC), time.clock_gettime_ns(time.CLOCK_BOOTTIME))]
    # Without composites the region is one render_passes call (the library
    # launches it in 32-pass launches): its matrix and seeds are staged before
    # the clock starts, so the region times the C-ABI calls, not their
    # argument conversion (~2.4 us of Python per call)
    first = 1 + a.warmup
    one_call = composite is None and F == 32
    if one_call:
        run = r.bind_render_passes(mvp, seeds[first:first + a.steps])
        sync = r.bind_synchronize()
    t0 = time.perf_counter()
    if one_call:
        run()
        launches = [min(32, a.steps - k) for k in range(0, a.steps, 32)]
    else:
        launches = passes(first, a.steps)
    if stamps:
        t_enq = time.perf_counter()
    if one_call:
        sync()
    else:
        r.synchronize()  # the march stream and (N > 1) the composite: the last all-reduce / composite is done
    el = time.perf_counter() - t0
    if stamps:
        clk.append((time.clock_gettime_ns(time.CLOCK_MONOTONIC), time.clock_gettime_ns(time.CLOCK_BOOTTIME)))
        Path(stamps).write_text(json.dumps({
            "rank": rank, "t0_perf": t0, "t_enq_perf": t_enq, "t_end_perf": t0 + el, "el_s": el,
            "monotonic_ns": [c[0] for c in clk], "boottime_ns": [c[1] for c in clk],
            "launches": None}))
    if multi:
        # the composite is on every rank's device; reading it back to the host
        # is the display's cost, not the pass's (done outside the timed region)
        r.read_composite()
        r.barrier()
    elif grouped:
        r.read_composite_all()  # the composite on devices[0] to the host, after the region
    kern_ms, n_launch = r.kernel_time()
    # timing only inside timed regions: launches between them are the library's
    # own (its macro-skip tuner times some of them itself, outside regions)
    r.enable_kernel_timing(False)
    macro = bool(r.last_launch().get("macro", False))  # the macro-cell bound in the timed launches
    if a.no_timing:
        kern_ms, n_launch = float("nan"), len(launches)
    assert n_launch == len(launches), (n_launch, len(launches))
    vals = np.array([el, kern_ms])
    if multi:
        vals = r.allreduce_host(vals, op="max")
    el_max, kern_ms_max = float(vals[0]), float(vals[1])

    photon_steps = world * group * R * R * S * a.steps
    value = photon_steps / el_max / 1e6
    # roofline of the march kernel: the algorithmic bytes its launches
    # materialise over the GPU time of the timed region, stamped by HIP events
    # on the renderer's stream (begin = the first launch's dispatch, end = a
    # marker behind the last launch); for equal launches this is bytes per
    # launch / average launch duration, the inter-launch gaps included
    # (conservative: rocprof's per-kernel average is slightly lower)
    alg_bytes = sum(cf.algorithmic_bytes_per_launch(R, S, n) for n in launches)
    achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
    kern_avg_ms = kern_ms_max / len(launches)
    bytes_per_launch = alg_bytes // len(launches)

    # the same workload at one launch per render() call (photon state stored and
    # reloaded every pass), continuing the pass sequence; N = 1 only
    # N > 1: the same march compositing after every pass (one launch + one RCCL
    # all-reduce of the (rgb*n, n) buffer per pass), bracketed like the main region
    per_pass = None
    if n_pp > 0:
        r.synchronize()
        if multi:
            r.barrier()
        t5 = time.perf_counter()
        passes(1 + a.warmup + a.steps, n_pp, F=1, every=1)
        r.synchronize()
        el5 = time.perf_counter() - t5
        if multi:
            r.read_composite()
            r.barrier()
            el5 = float(r.allreduce_host(np.array([el5, 0.0]), op="max")[0])
        else:
            r.read_composite_all()
        per_pass = {"value": round(world * group * R * R * S * n_pp / el5 / 1e6, 3),
                    "ms_per_step": round(el5 * 1e3 / n_pp, 5), "steps": n_pp,
                    "note": ("one march launch and one RCCL all-reduce of the R^2 float4 (rgb*n, n) "
                             "buffer per pass (north_star's per-pass composite)") if multi else
                            (f"one march launch per GPU and one device-list composite ({a.transport}) "
                             "per pass (north_star's per-pass composite)")}

    unfused = None
    if n_unfused > 0:
        # one-pass launches before the region, as a display loop runs them (the
        # library's macro-skip tuner measures this launch size here, untimed)
        passes(1 + a.warmup + a.steps + n_unfused + n_api + n_pp, n_uwarm, F=1)
        r.synchronize()
        r.enable_kernel_timing(not a.no_timing)  # restart the launch timings
        t1 = time.perf_counter()
        ul = passes(1 + a.warmup + a.steps, n_unfused, F=1)
        r.synchronize()
        el1 = time.perf_counter() - t1
        uk_ms, un = r.kernel_time()
        r.enable_kernel_timing(False)
        if a.no_timing:
            uk_ms, un = float("nan"), len(ul)
        assert un == len(ul)
        ub = cf.algorithmic_bytes_per_launch(R, S, 1)
        ua = ub * un / (uk_ms * 1e-3) / 1e9
        unfused = {"value": round(R * R * S * n_unfused / el1 / 1e6, 3),
                   "ms_per_step": round(el1 * 1e3 / n_unfused, 5), "steps": n_unfused,
                   "kernel_avg_us": round(uk_ms * 1e3 / un, 3),
                   "achieved": round(ua, 1), "frac": round(ua / HBM_PEAK_GBPS, 4),
                   "algorithmic_bytes_per_launch": ub}

    # the drop-in path: one vptmcm_render() call per pass, as the JS renderer's
    # render() makes them; the library queues them and launches fused marches
    render_api = None
    if n_api > 0:
        r.synchronize()
        first = 1 + a.warmup + a.steps + n_unfused
        t2 = time.perf_counter()
        for k in range(n_api):
            r.render(mvp, seeds[first + k])
        r.synchronize()
        el2 = time.perf_counter() - t2
        render_api = {"value": round(R * R * S * n_api / el2 / 1e6, 3),
                      "ms_per_step": round(el2 * 1e3 / n_api, 5), "steps": n_api,
                      "note": "one render() call per pass through the C-ABI (ctypes); the "
                              "library fuses queued passes into multi-pass launches"}

    # The volume-filling regime: the golden 'near' camera puts
    # the volume in front of every pixel, so every photon-step is an in-volume
    # gather; same volume, TF, bins and launch shape as the main line
    near = None
    if a.near_steps > 0 and single and a.camera == "default":
        r.synchronize()
        mn = cf.golden_mvp("near")
        nseeds = cf.seed_stream(a.near_steps + 321, start=3, rank=rank)
        r.reset(mn, nseeds[0])
        # the photons' depth distribution and the deal settle; ten launches also
        # give the library's macro-skip tuner its pairs for this camera
        r.render_passes(mn, nseeds[1:321])
        r.synchronize()
        r.enable_kernel_timing(not a.no_timing)
        t6 = time.perf_counter()
        nl = passes_on(nseeds, 321, a.near_steps, m=mn)
        r.synchronize()
        el6 = time.perf_counter() - t6
        nk_ms, nn = r.kernel_time()
        r.enable_kernel_timing(False)
        nmacro = bool(r.last_launch().get("macro", False))
        nbytes = sum(cf.algorithmic_bytes_per_launch(R, S, n) for n in nl)
        nshapes = sorted(set(nl))
        # the same region with the macro-cell bound switched off (what the march
        # costs here without it; the line above keeps the library's choice)
        nk_off = None
        if not a.no_timing and nmacro:
            r.set_macro_skip("off")
            r.render_passes(mn, nseeds[1:33])  # one launch at the new setting, untimed
            r.synchronize()
            r.enable_kernel_timing(True)
            passes_on(nseeds, 321, a.near_steps, m=mn)
            r.synchronize()
            nk_off, _ = r.kernel_time()
            r.enable_kernel_timing(False)
            r.set_macro_skip(os.environ.get("VPTMCM_MAJ", "auto") if os.environ.get("VPTMCM_MAJ") in
                             ("on", "off", "auto") else "auto")
        near = {"value": round(R * R * S * a.near_steps / el6 / 1e6, 3),
                "ms_per_step": round(el6 * 1e3 / a.near_steps, 5), "steps": a.near_steps,
                "passes_per_launch": nshapes[0] if len(nshapes) == 1 else nshapes,
                "kernel_us_per_pass": None, "roofline": None, "gather_roofline": None,
                "macro_skip": nmacro,
                "kernel_us_per_pass_bound_off": (round(nk_off * 1e3 / a.near_steps, 3) if nk_off else None),
                "workload": "same volume, TF, bins and launch shape as the main line with the golden "
                            "'near' camera: the volume fills the frame, every photon-step gathers"}
        if not a.no_timing:
            nach = nbytes / (nk_ms * 1e-3) / 1e9
            near["kernel_us_per_pass"] = round(nk_ms * 1e3 / a.near_steps, 3)
            near["roofline"] = {"bound": "hbm", "achieved": round(nach, 1), "peak": HBM_PEAK_GBPS,
                                "unit": "GB/s", "frac": round(nach / HBM_PEAK_GBPS, 4),
                                "algorithmic_bytes_per_launch": nbytes // len(nl), "traffic": None}
            ne = pmc_entry(a, R, S, nshapes, "near", nmacro)
            if ne is not None:
                launch_s = nk_ms * 1e-3 / nn
                fills = ne["read_requests"]["128B"] + ne["read_requests"]["64B"] + ne["read_requests"]["32B"]
                near["roofline"].update({
                    "traffic": ne["hbm_bytes_per_launch"], "traffic_source": ne["_source"],
                    "traffic_gbps": round(ne["hbm_bytes_per_launch"] / launch_s / 1e9, 1),
                    "traffic_frac": round(ne["hbm_bytes_per_launch"] / launch_s / 1e9 / HBM_PEAK_GBPS, 4)})
                gp = ne.get("_gather_peak") or {}
                if gp.get("ggathers_per_s"):
                    g = fills / launch_s / 1e9
                    near["gather_roofline"] = {
                        "bound": "scattered 8-B gathers (one 128-B L2 fill each)", "achieved": round(g, 2),
                        "peak": gp["ggathers_per_s"], "unit": "G gathers/s",
                        "frac": round(g / gp["ggathers_per_s"], 4), "peak_source": gp.get("source"),
                        "fills_per_launch": fills, "fills_source": ne["_source"]}
                if ne.get("issue"):
                    iv = ne["issue"]
                    ach = iv["valu_insts"] / launch_s / 1e9
                    near["issue"] = {"bound": "valu-issue", "achieved": round(ach, 1), "peak": VALU_PEAK_G,
                                     "unit": "G wave-instructions/s", "frac": round(ach / VALU_PEAK_G, 4),
                                     "valu_per_photon_step": iv["valu_per_photon_step"]}

    # The launch shape that actually ran (the last launch of a region can be
    # shorter than --fuse, and --steps < --fuse gives one short launch).
    shapes = sorted(set(launches))
    ppl = shapes[0] if len(shapes) == 1 else shapes
    # PMC-derived memory-side bytes per launch (profiles/): attached only when a
    # profile of this exact launch shape (R, S, layout, volume, passes) exists.
    traffic, traffic_src, issue = None, None, None
    e = pmc_entry(a, R, S, shapes, a.camera, macro)
    if e is not None:
        traffic = e.get("hbm_bytes_per_launch")
        traffic_src = e["_source"]
        # VALU issue roofline: the launch's VALU wave-instructions (PMC, same
        # launch shape) over its live duration, against 1024 SIMD-32s issuing
        # one wave64 VALU instruction per 2 cycles at the 2.4 GHz peak clock
        iv = e.get("issue")
        if iv and not a.no_timing:
            ach = iv["valu_insts"] / (kern_avg_ms * 1e-3) / 1e9
            issue = {"bound": "valu-issue", "achieved": round(ach, 1),
                     "peak": VALU_PEAK_G, "unit": "G wave-instructions/s",
                     "frac": round(ach / VALU_PEAK_G, 4),
                     "valu_per_photon_step": iv["valu_per_photon_step"],
                     "source": traffic_src}

    # The march on a UI-like configuration of the same volume: 8 uneven bins and
    # a materials TF with wavelength-varying anisotropy (MODE 6: FAST geometry,
    # the TF's distinct rows and the exact wavelength-bin table in LDS)
    general = None
    if a.general_steps > 0 and single:
        r.synchronize()
        r.set_material_tf(cf.tf_materials(True))
        r.set_spectrum(cf.spectrum_buffer("8_uneven"))
        gseeds = cf.seed_stream(a.general_steps + 33, start=1, rank=rank)
        r.reset(mvp, gseeds[0])
        r.render_passes(mvp, gseeds[1:33])
        r.synchronize()
        r.enable_kernel_timing(not a.no_timing)
        t3 = time.perf_counter()
        gl = passes_on(gseeds, 33, a.general_steps)
        r.synchronize()
        el3 = time.perf_counter() - t3
        gk_ms, gn = r.kernel_time()
        r.enable_kernel_timing(False)
        general = {"value": round(R * R * S * a.general_steps / el3 / 1e6, 3),
                   "ms_per_step": round(el3 * 1e3 / a.general_steps, 5),
                   "steps": a.general_steps, "passes_per_launch": sorted(set(gl)),
                   "kernel_us_per_pass": (round(gk_ms * 1e3 / a.general_steps, 3)
                                          if not a.no_timing else None),
                   "workload": "same volume/camera, tf_materials(varying anisotropy), "
                               "8_uneven bins: a UI-like TF (row-deduplicated in LDS) and "
                               "uneven bins (exact bin table in LDS), march MODE 6 (MODE 2 is the "
                               "headline's)"}

    # The RGB sibling ('mcm-compute') on the same volume and camera:
    # a 256 x 1 sRGB TF ramp, HG anisotropy 0.7, white 1x1 environment
    rgb = None
    if a.rgb_steps > 0 and single:
        r.synchronize()
        q = vptmcm.Renderer(R, device=device, layout=layout, renderer=vptmcm.RENDERER_RGB)
        x = np.arange(256)
        ttf = np.zeros((1, 256, 4), np.uint8)
        ttf[0, :, 0], ttf[0, :, 1], ttf[0, :, 2] = 255 - x // 2, 128 + x // 4, x
        ttf[0, :, 3] = np.clip((x - 40) * 2, 0, 255)
        q.set_volume(vol)
        q.set_transfer_function(ttf)
        q.set_environment((255, 255, 255, 255))
        q.set_params(extinction=a.extinction, anisotropy=0.7, bounces=8, steps=S)
        rseeds = cf.seed_stream(a.rgb_steps + 321, start=2, rank=rank)
        q.reset(mvp, rseeds[0])
        for k in range(10):  # settle; the macro-skip tuner's pairs for this renderer
            q.render_passes(mvp, rseeds[1 + 32 * k:33 + 32 * k])
        q.synchronize()
        q.enable_kernel_timing(not a.no_timing)
        t4 = time.perf_counter()
        done = 0
        while done < a.rgb_steps:
            n = min(F, a.rgb_steps - done)
            q.render_passes(mvp, rseeds[321 + done:321 + done + n])
            done += n
        q.synchronize()
        el4 = time.perf_counter() - t4
        qk_ms, _ = q.kernel_time()
        q.enable_kernel_timing(False)
        rmacro = bool(q.last_launch().get("macro", False))
        rgb = {"value": round(R * R * S * a.rgb_steps / el4 / 1e6, 3),
               "ms_per_step": round(el4 * 1e3 / a.rgb_steps, 5), "steps": a.rgb_steps,
               "kernel_us_per_pass": (round(qk_ms * 1e3 / a.rgb_steps, 3)
                                      if not a.no_timing else None),
               "macro_skip": rmacro,
               "workload": "RGB sibling renderer (MCMComputeRenderer.wgsl) on the same volume and "
                           "camera: 256x1 sRGB TF ramp, anisotropy 0.7, white environment"}
        q.close()

    r.synchronize()
    js_api = None
    if a.js_steps > 0 and single and a.tf == "spectral" and a.camera == "default":
        js_api = js_api_line(vol, tf, spec, R, S, a.extinction, a.js_steps, a.settle_ms)

    n_gpus = world * group
    if multi:
        parallelism = (f"photon-parallel replicas x{world}, one process per GPU, RCCL "
                       + ("reduce-scatter (summed frame kept sharded over the ranks)"
                          if a.shard_composite == "on" else "all-reduce")
                       + f" of (rgb*n, n) every {every} pass(es)")
        comp_kind = "rccl-reduce-scatter" if a.shard_composite == "on" else "rccl-allreduce"
    elif grouped:
        parallelism = (f"photon-parallel replicas x{group} in one process (device-list handle over "
                       f"devices {devs}), composite of (rgb*n, n) every {every} pass(es)"
                       + (", each device compositing its 1/N pixel shard over xGMI peer reads"
                          if a.transport == "peer" else f", reduced to device {devs[0]}"))
        comp_kind = {"peer": "peer-sharded", "rccl": "rccl-reduce"}[a.transport]
    else:
        parallelism, comp_kind = "single GPU", None
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mphoton-steps/s",
            "n_gpus": n_gpus, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el_max * 1e3 / a.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {
                "workload": (f"{config_name(a.volume, n_gpus)}: {a.volume}^3 fBm volume (seed "
                             f"{volume_seed(a.volume)})" if a.volume_kind == "fbm" else
                             f"custom: {a.volume}^3 two-spheres volume (generate_test_volume.ipynb)")
                            + f", {TF_DESC.get(a.tf, a.tf + ' TF')}, R={R}, S={S}, "
                            f"{a.bins} bins, extinction {a.extinction}, "
                            + (f"{a.camera} camera" if a.camera_mix is None else
                               f"camera mix {a.camera_mix} (default -> near)"),
                "resolution": R, "photon_steps_per_pass": S, "volume": a.volume,
                "volume_layout": a.layout, "passes_per_launch": ppl,
                "clock_settle_ms": round(settle_ms, 1), "clock_settle_passes": settle_passes,
                "parallelism": parallelism,
                "composite_transport": comp_kind,
                "devices": devs if grouped else None,
                # the macro-cell alpha bound (VPTMCM_MAJ, default auto: the library's
                # tuner measures it on and off and keeps the faster) in the timed launches
                "macro_skip": macro,
            },
            "hbm_gbps_algorithmic": round(achieved, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_ratio": (round(traffic / bytes_per_launch, 2) if traffic else None),
                         # the same PMC bytes over this run's launch time: L2-miss line
                         # traffic (128-B fills; Infinity Cache hits included) per second
                         "traffic_gbps": (round(traffic / (kern_avg_ms * 1e-3) / 1e9, 1)
                                          if traffic and not a.no_timing else None),
                         "traffic_frac": (round(traffic / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                          if traffic and not a.no_timing else None),
                         "issue": issue,
                         "kernel": "k_march", "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
                         # host wall time of the timed region minus its march GPU time (launch
                         # enqueue, dispatch, completion wake-up)
                         "region_wall_us": round(el_max * 1e6, 1),
                         "wall_minus_kernel_us": (round(el_max * 1e6 - kern_ms_max * 1e3, 1)
                                                  if not a.no_timing else None),
                         "passes_per_launch": ppl,
                         "kernel_us_per_pass": round(kern_ms_max * 1e3 / a.steps, 3),
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         # SURVEY 8(d)'s per-unit figure (31.0 B per photon-step at
                         # nb = 12, S = 8: the reference materialises the photon
                         # state and the image every pass) x the photon-steps of the
                         # timed region, over the same GPU time; `frac` above counts
                         # only the bytes this build's fused launches materialise
                         "per_unit": {
                             "bytes_per_photon_step": round(cf.algorithmic_bytes_per_pass(R, S) / (R * R * S), 2),
                             "achieved": round(cf.algorithmic_bytes_per_pass(R, S) * a.steps
                                               / (kern_ms_max * 1e-3) / 1e9, 1),
                             "frac": round(cf.algorithmic_bytes_per_pass(R, S) * a.steps
                                           / (kern_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}},
            "unfused": unfused,
            "render_api": render_api,
            "js_api": js_api,
            "general": general,
            "near": near,
            "rgb": rgb,
            "per_pass_allreduce": per_pass,
            "cpu_baseline": None,
            "volume_gen_s": round(gen_s, 2),
        }
        if n_gpus == 1 and a.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(vol, tf, spec, spd, ldir, mvp, R, S, a.extinction,
                                               a.cpu_seconds)
        print(json.dumps(out), flush=True)
    r.close()


def entry() -> None:
    try:
        main()
    except rendezvous.RendezvousError:
        # a peer never reached the rendezvous: no communicator exists, so the
        # process ends normally with the communicator failure's exit code
        import traceback
        traceback.print_exc()
        sys.exit(3)
    except vptmcm.VptError as e:
        if e.code != vptmcm.ECOMM:
            raise
        # a failed RCCL communicator (a peer rank died mid-run): report and end
        # the process at once — RCCL's own threads still blocked on the dead
        # peer must not hold up interpreter shutdown
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(3)


if __name__ == "__main__":
    entry()
