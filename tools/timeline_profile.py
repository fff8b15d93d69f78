#!/usr/bin/env python3
"""Timeline of a march launch, per wave (experiment build, never the product).

Runs the bench workload (C3) on build/variants/libvptmcm_<variant>.so built with
-DVPT_STAMP=2 (tools/variants.py tl='-DVPT_STAMP=2'): every wave writes the
100 MHz s_memrealtime at five points of the launch into the fp32 image buffer
(csrc/stamp.h): entry, tile scheduled, LDS filled + photon state resident, pass
loop done, stores complete. For one-pass and fused launches it reports, over
the waves (times relative to the launch's first wave entry, µs):

  entry spread      when the waves start (the dispatch ramp)
  schedule          entry -> tile known
  fill              tile known -> LDS TF + photon state resident
  passes            the pass loop (volume / background waves, by SIMD load)
  store             the end-of-launch state, image and flag stores
  span              first entry -> last store, against the launch's event time

    VPTMCM_LIB=tl python tools/timeline_profile.py [--passes 1 20 32]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402


def q(x):
    x = np.asarray(x, np.float64)
    if x.size == 0:
        return None
    return {"min": round(float(x.min()), 2), "med": round(float(np.median(x)), 2),
            "p90": round(float(np.percentile(x, 90)), 2), "max": round(float(x.max()), 2)}


def reduce(w, ev_us):
    live = w[:, 0] != 0
    w = w[live]
    t = w[:, :5].astype(np.int64)
    t0 = t[:, 0].min()
    t = (t - t0) & 0xFFFFFFFF  # 32-bit wrap of the 100 MHz counter
    t = t.astype(np.float64) / 100.0  # µs
    vol = (w[:, 5] & 0xFF) == 1
    hw, xcc = w[:, 7], (w[:, 5] >> 8) & 0xFF
    simd = (xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) | \
        (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    ids, cnt = np.unique(simd[vol], return_counts=True)
    load = dict(zip(ids.tolist(), cnt.tolist()))
    nl = np.array([load.get(int(s), 0) for s in simd])
    out = {"waves": int(len(w)), "volume_waves": int(vol.sum()),
           "event_us": round(ev_us, 2), "span_us": round(float(t[:, 4].max()), 2),
           "entry": q(t[:, 0]), "entry_xcd_first": {int(x): round(float(t[xcc == x, 0].min()), 2)
                                                    for x in np.unique(xcc)},
           "schedule": q(t[:, 1] - t[:, 0]), "fill": q(t[:, 2] - t[:, 1]),
           "fill_end": q(t[:, 2]),
           "passes_volume": q(t[vol, 3] - t[vol, 2]), "passes_background": q(t[~vol, 3] - t[~vol, 2]),
           "store": q(t[:, 4] - t[:, 3]),
           "end_volume": q(t[vol, 4]), "end_background": q(t[~vol, 4])}
    for k in sorted(set(nl[vol].tolist())):
        s = vol & (nl == k)
        out[f"volume_simd_load{k}"] = {"passes": q(t[s, 3] - t[s, 2]), "end": q(t[s, 4])}
    # the last wave: where its time went
    if (w[:, 6] != 0).all():  # -DVPT_TL_PROBE=1: the TF copy's landing time in word 6
        t6 = ((w[:, 6].astype(np.int64) - t0) & 0xFFFFFFFF).astype(np.float64) / 100.0
        out["probe_tf_copy"] = q(t6 - t[:, 0])
        out["probe_schedule_after_copy"] = q(t[:, 1] - t6)
    j = int(np.argmax(t[:, 4]))
    out["last_wave"] = {"volume": bool(vol[j]), "simd_load": int(nl[j]),
                        "marks_us": [round(float(v), 2) for v in t[j]]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, nargs="+", default=[1, 20, 32])
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--volume", type=int, default=512)
    ap.add_argument("--dump", default="", help="save every launch's raw records (npz)")
    a = ap.parse_args()
    R, S = 512, 8
    r = vptmcm.Renderer(R, device=0, layout=vptmcm.LAYOUT_CORNER8)
    r.set_volume(cf.fbm_volume(a.volume, 512 if a.volume == 512 else a.volume))
    r.set_material_tf(cf.tf_spectral())
    spd, ldir = cf.light_default()
    r.set_light(spd, ldir)
    r.set_spectrum(cf.spectrum_buffer("12"))
    r.set_params(extinction=32.0, bounces=8, steps=S)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(64, start=0)
    r.reset(mvp, seeds[0])
    for _ in range(300):  # ~150 ms of fused launches: clock settled
        r.render_passes(mvp, seeds[1:33])
    r.synchronize()
    res = {"workload": "C3 512^3 corner8, R=512, S=8", "launch": {}}
    raw = {}
    for F in a.passes:
        runs = []
        for k in range(a.samples):
            r.render_passes(mvp, seeds[1:33])  # keep the clock up between samples
            r.synchronize()
            r.enable_kernel_timing(True)
            r.render_passes(mvp, seeds[1 + (k % 8):1 + (k % 8) + F])
            ms, n = r.kernel_time()
            r.enable_kernel_timing(False)
            w = r.read_rgb().reshape(-1).view(np.uint32)[: (R * R // 64) * 8].reshape(-1, 8).copy()
            runs.append(reduce(w, ms * 1e3))
            raw[f"F{F}_{k}"] = w
        med = sorted(runs, key=lambda d: d["span_us"])[len(runs) // 2]
        med["event_us_all"] = [d["event_us"] for d in runs]
        med["span_us_all"] = [d["span_us"] for d in runs]
        res["launch"][str(F)] = med
    r.close()
    if a.dump:
        np.savez_compressed(a.dump, **raw)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
