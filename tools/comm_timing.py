#!/usr/bin/env python3
"""Host-side timing of every call of the N > 1 composite path with one rank
(analysis): where the wall time of a timed region with all-reduces goes.

    python tools/comm_timing.py [--passes 32] [--reps 6]
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
    ap.add_argument("--passes", type=int, default=32)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    r = vptmcm.Renderer(512, device=0)
    r.set_volume(cf.fbm_volume(512, 512))
    r.set_material_tf(cf.tf_spectral())
    r.set_light(*cf.light_default())
    r.set_spectrum(cf.spectrum_buffer("12"))
    r.set_params(extinction=32.0, bounces=8, steps=8)
    t = time.perf_counter()
    r.comm_init(vptmcm.unique_id(), 1, 0)
    init_ms = (time.perf_counter() - t) * 1e3
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(a.passes + 1, start=0)
    r.reset(mvp, seeds[0])
    rows = []
    for k in range(a.reps):
        t0 = time.perf_counter()
        r.render_passes(mvp, seeds[1:1 + a.passes])
        t1 = time.perf_counter()
        r.allreduce_radiance()
        t2 = time.perf_counter()
        r.synchronize()
        t3 = time.perf_counter()
        r.read_composite()
        t4 = time.perf_counter()
        r.barrier()
        t5 = time.perf_counter()
        rows.append([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4])
    r.close()
    m = np.median(np.array(rows) * 1e6, axis=0)
    print(json.dumps({"comm_init_ms": round(init_ms, 1), "passes": a.passes,
                      "first_rep_us": [round(x * 1e6, 1) for x in rows[0]],
                      "median_us": dict(zip(["render_passes", "allreduce_radiance", "synchronize",
                                             "read_composite", "barrier"], [round(float(x), 1) for x in m]))}))


if __name__ == "__main__":
    main()
