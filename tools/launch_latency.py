#!/usr/bin/env python3
"""Where the wall time of a short timed region goes (the driver's --steps 20):
host enqueue of one 20-pass launch, the launch's GPU time (HIP events), and the
synchronize, over repeated regions after clock settling. Analysis only.

    python tools/launch_latency.py [--passes 20] [--regions 30]
(env VPTMCM_SYNC_SPIN=1: spin-waiting host synchronisation; --no-timing: no HIP events)
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--regions", type=int, default=30)
    ap.add_argument("--no-timing", action="store_true", help="no HIP events in the region")
    a = ap.parse_args()
    r = vptmcm.Renderer(512, device=0)
    r.set_volume(cf.fbm_volume(512, 512))
    r.set_material_tf(cf.tf_spectral())
    spd, ldir = cf.light_default()
    r.set_light(spd, ldir)
    r.set_spectrum(cf.spectrum_buffer("12"))
    r.set_params(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(32, start=0)
    r.reset(mvp, seeds[0])
    t = time.perf_counter()
    while time.perf_counter() - t < 0.2:
        for _ in range(8):
            r.render_passes(mvp, seeds[1:33])
        r.synchronize()
    sd = seeds[1:1 + a.passes]
    enq, syn, wall, kern = [], [], [], []
    for _ in range(a.regions):
        r.synchronize()
        r.enable_kernel_timing(not a.no_timing)
        t0 = time.perf_counter()
        r.render_passes(mvp, sd)
        t1 = time.perf_counter()
        r.synchronize()
        t2 = time.perf_counter()
        k_ms = r.kernel_time()[0] if not a.no_timing else float("nan")
        enq.append((t1 - t0) * 1e6)
        syn.append((t2 - t1) * 1e6)
        wall.append((t2 - t0) * 1e6)
        kern.append(k_ms * 1e3)
    r.close()
    med = lambda v: round(float(np.median(v)), 2)  # noqa: E731
    print(json.dumps({"passes": a.passes, "timing": not a.no_timing, "enqueue_us": med(enq), "sync_us": med(syn),
                      "wall_us": med(wall), "kernel_region_us": med(kern),
                      "overhead_us": round(med(wall) - med(kern), 2),
                      # the first region is the one a single-region bench (the driver's) times
                      "first": {"enqueue_us": round(enq[0], 2), "sync_us": round(syn[0], 2),
                                "wall_us": round(wall[0], 2), "kernel_region_us": round(kern[0], 2)},
                      "wall_us_max": round(max(wall), 2), "wall_us_min": round(min(wall), 2)}))


if __name__ == "__main__":
    main()
