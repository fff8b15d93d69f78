#!/usr/bin/env python3
"""Is the driver line's run-to-run spread a property of the allocation? Within
one process, create the renderer (fresh photon / volume / table allocations)
several times and time the driver's region shape (one 20-pass launch) on each:
if the per-renderer medians spread like separate processes do (302-336 us), the
placement of the buffers decides; if they agree, the spread comes from outside
the allocation (clock state). Analysis only.

    python tools/alloc_var.py [--trials 6] [--regions 12] [--passes 20]
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
    ap.add_argument("--trials", type=int, default=6)
    ap.add_argument("--regions", type=int, default=12)
    ap.add_argument("--passes", type=int, default=20)
    a = ap.parse_args()
    vol = cf.fbm_volume(512, 512)
    tf = cf.tf_spectral()
    spd, ldir = cf.light_default()
    spec = cf.spectrum_buffer("12")
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(33, start=0)
    keep = []  # renderers kept alive so each trial's buffers land elsewhere
    for t in range(a.trials):
        r = vptmcm.Renderer(512, device=0)
        r.set_volume(vol)
        r.set_material_tf(tf)
        r.set_light(spd, ldir)
        r.set_spectrum(spec)
        r.set_params(extinction=32.0, bounces=8, steps=8)
        r.reset(mvp, seeds[0])
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.15:
            for _ in range(8):
                r.render_passes(mvp, seeds[1:33])
            r.synchronize()
        kern, wall = [], []
        for _ in range(a.regions):
            r.synchronize()
            r.enable_kernel_timing(True)
            w0 = time.perf_counter()
            r.render_passes(mvp, seeds[1:1 + a.passes])
            r.synchronize()
            wall.append((time.perf_counter() - w0) * 1e6)
            kern.append(r.kernel_time()[0] * 1e3)
        print(json.dumps({"trial": t, "kernel_us_median": round(float(np.median(kern)), 2),
                          "kernel_us_min": round(min(kern), 2), "kernel_us_max": round(max(kern), 2),
                          "first_kernel_us": round(kern[0], 2),
                          "wall_us_median": round(float(np.median(wall)), 2)}), flush=True)
        keep.append(r)
    for r in keep:
        r.close()


if __name__ == "__main__":
    main()
