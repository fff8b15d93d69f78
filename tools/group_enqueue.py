#!/usr/bin/env python3
"""Host enqueue cost of a device-list handle's forwarded launch, with and
without the per-replica worker threads (VPTMCM_GROUP_THREADS=0).

N replicas on device 0 (devices = [0] * N, the only way to drive a group on a
one-GPU box): the call's host duration is what the caller's thread spends
forwarding one 32-pass render_passes to every replica, i.e. the bound on the
skew between the first and the last replica's launch on an N-GPU node (the
kernels themselves serialise on the one GPU here and are not the measurement).
With --composite, every render_passes is followed by composite() (the
driver-shaped region of a device-list bench: one composite per launch), whose
host duration is reported too: the sharded PEER composite's enqueue (pack,
shard kernels, events on every replica's threads) happens while the 32-pass
march runs, so it is hidden behind it when render_passes + composite return
well before the march ends. Run under rocprofv3 --kernel-trace to get the
device chain from the last march to the last shard kernel
(tools/composite_trace.py).
Prints one JSON line per (N, threads).

    python tools/group_enqueue.py [--ns 2 4 8] [--reps 40] [--composite]
"""
import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "vpt-spectral-volume-rendering_amd" / "python"))

import numpy as np  # noqa: E402

import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402


def case(n, threads, vol, reps, composite=False):
    os.environ["VPTMCM_GROUP_THREADS"] = "1" if threads else "0"
    g = vptmcm.Renderer(512, devices=[0] * n, layout=vptmcm.LAYOUT_COLUMN4)
    g.set_spectrum(cf.spectrum_buffer("12"))
    g.set_volume(vol)
    g.set_material_tf(cf.tf_spectral())
    g.set_light(np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32))
    g.set_params(extinction=100.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    g.reset(mvp, 1)
    seeds = cf.seed_stream(32, start=2)
    enq, comp, wall = [], [], []
    for k in range(reps + 5):
        g.synchronize()
        t0 = time.perf_counter()
        g.render_passes(mvp, seeds)
        t1 = time.perf_counter()
        if composite:
            g.composite()
        tc = time.perf_counter()
        g.synchronize()
        t2 = time.perf_counter()
        if k >= 5:
            enq.append((t1 - t0) * 1e6)
            comp.append((tc - t1) * 1e6)
            wall.append((t2 - t0) * 1e6)
    # ingest of the same volume (one GPU: the copies share its link)
    t0 = time.perf_counter()
    g.set_volume(vol)
    g.synchronize()
    ingest_ms = (time.perf_counter() - t0) * 1e3
    g.close()
    return {"n": n, "threads": threads, "enqueue_us_median": round(statistics.median(enq), 1),
            "enqueue_us_p90": round(sorted(enq)[int(0.9 * len(enq))], 1),
            "composite_enqueue_us_median": round(statistics.median(comp), 1) if composite else None,
            "composite_enqueue_us_p90": round(sorted(comp)[int(0.9 * len(comp))], 1) if composite else None,
            "wall_us_median": round(statistics.median(wall), 1), "ingest_ms": round(ingest_ms, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--volume", type=int, default=256)
    ap.add_argument("--composite", action="store_true")
    ap.add_argument("--threads", choices=["both", "on", "off"], default="both")
    a = ap.parse_args()
    vol = cf.fbm_volume(a.volume, 7)
    for n in a.ns:
        arms = {"both": (False, True, False, True), "on": (True,), "off": (False,)}[a.threads]
        for threads in arms:  # alternating pairs
            print(json.dumps(case(n, threads, vol, a.reps, a.composite)), flush=True)


if __name__ == "__main__":
    main()
