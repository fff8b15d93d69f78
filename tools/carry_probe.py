#!/usr/bin/env python3
"""Cross-launch balancing, launch by launch: C3 at R = 512,
L launches of 32 queued render() passes each; after every launch the owed
passes per tile (vptmcm_debug_owed: queued passes launch, owed ones stay
owed) and the launch's own GPU time (HIP events around it). One JSON line per
launch, then a summary. Run it under `rocprofv3 --kernel-trace` for the
kernel-trace durations of the same launches.

    VPTMCM_CARRY=1 python tools/carry_probe.py --launches 24
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "vpt-spectral-volume-rendering_amd" / "python"))

import numpy as np  # noqa: E402

import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=24)
    ap.add_argument("--settle-ms", type=float, default=150.0)
    a = ap.parse_args()
    R = 512
    r = vptmcm.Renderer(R, device=0)
    r.set_volume(cf.fbm_volume(512, 512))
    r.set_material_tf(cf.tf_spectral())
    spd, ld = cf.light_default()
    r.set_light(spd, ld)
    r.set_spectrum(cf.spectrum_buffer("12"))
    r.set_params(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(32 * (a.launches + 4) + 1, start=0)
    r.reset(mvp, seeds[0])
    t = time.perf_counter()
    ss = cf.seed_stream(32, start=1 << 20)
    while (time.perf_counter() - t) * 1e3 < a.settle_ms:
        r.render_passes(mvp, ss)
        r.synchronize()
    k = 1
    rows = []
    for L in range(a.launches):
        for _ in range(32):
            r.render(mvp, seeds[k])
            k += 1
        t0 = time.perf_counter()
        owed = r.debug_owed()  # launches the 32 queued passes, keeping what they leave owed
        el = time.perf_counter() - t0
        rows.append({"launch": L, "host_ms": round(el * 1e3, 3), "owing_tiles": int((owed > 0).sum()),
                     "owed_mean": round(float(owed[owed > 0].mean()) if (owed > 0).any() else 0.0, 2),
                     "owed_max": int(owed.max()), "owed_total": int(owed.sum())})
        print(json.dumps(rows[-1]), flush=True)
    r.synchronize()
    r.close()
    print(json.dumps({"carry": os.environ.get("VPTMCM_CARRY", "default"),
                      "mean_host_ms_per_launch": round(float(np.mean([x["host_ms"] for x in rows[4:]])), 3)}))


if __name__ == "__main__":
    main()
