#!/usr/bin/env python3
"""Diagnostics of the device-list composite against oracle replicas
(measurement aid): for a few (R, replicas, layout, fuzz case) settings, how
many pixels of the composite's counts / fp32 image differ, and what the
differing values look like (got vs the oracle composite, vs the composite of
fewer passes). One JSON line per setting.

    python tools/group_debug.py
"""
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "vpt-spectral-volume-rendering_amd" / "python", REPO / "oracle", REPO / "tests"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402

import oracle as orc  # noqa: E402
import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402

from test_gpu_group import _composite  # noqa: E402


def oracle_reps(R, vol, spec, tf, spd, ld, params, mvp, start, n_rep, n_seeds):
    reps = []
    for j in range(n_rep):
        o = orc.Oracle(R)
        o.set_spectrum(spec)
        o.volume, o.tf, o.light, o.light_dir = vol, tf, spd, ld
        o.params.update(**params)
        rs = cf.seed_stream(n_seeds, start=start, rank=j)
        o.reset(mvp, rs[0], nthreads=16)
        rgb = None
        for s_ in rs[1:]:
            rgb, _ = o.render(mvp, s_, nthreads=16)
        reps.append((o, rgb))
    return reps


def case(name, R, vol, spec, tf, spd, ld, params, mvp, layout, n_rep, start, mid_read=True):
    seeds = cf.seed_stream(5, start=start)
    out = {"case": name, "R": R, "n_rep": n_rep, "layout": layout,
           "threads": os.environ.get("VPTMCM_GROUP_THREADS", "1")}
    with vptmcm.Renderer(R, devices=[0] * n_rep, layout=layout) as g:
        g.set_spectrum(spec)
        g.set_volume(vol)
        g.set_material_tf(tf)
        g.set_light(spd, ld)
        g.set_params(**params)
        g.reset(mvp, seeds[0])
        g.render(mvp, seeds[1])
        if mid_read:
            mid = g.read_composite_all()
        g.render_passes(mvp, seeds[2:])
        q, crgb, n = g.read_composite_all()
    want = _composite(oracle_reps(R, vol, spec, tf, spd, ld, params, mvp, start, n_rep, 5))
    w1 = _composite(oracle_reps(R, vol, spec, tf, spd, ld, params, mvp, start, n_rep, 2))
    bad_n = ~(n == want[2])
    out["bad_counts"] = int(bad_n.sum())
    out["bad_rgb_words"] = int((~(crgb.view(np.uint32) == want[0].view(np.uint32))).sum())
    if bad_n.any():
        idx = np.argwhere(bad_n)[:6]
        out["sample"] = [{"px": [int(a) for a in i], "got": float(n[tuple(i)]), "want": float(want[2][tuple(i)]),
                          "want_after_1_pass": float(w1[2][tuple(i)])} for i in idx]
        out["counts_equal_1_pass_composite"] = bool(np.array_equal(n, w1[2]))
        out["bad_rows"] = sorted({int(i[0]) for i in np.argwhere(bad_n)})[:32]
    if mid_read:
        out["mid_counts_ok"] = bool(np.array_equal(mid[2], w1[2]))
    print(json.dumps(out), flush=True)


def main():
    from test_gpu_fuzz import _draw, _volume
    R, shape, layout, spec, tf, ld, spd, params, mvp, vol_seed, what = _draw(400)
    vol = _volume(shape, vol_seed)
    for n_rep in (6, 2):
        case(f"fuzz400 {what}", R, vol, spec, tf, spd, ld, params, mvp, layout, n_rep, 9)
    case("fuzz400 no mid read", R, vol, spec, tf, spd, ld, params, mvp, layout, 6, 9, mid_read=False)
    os.environ["VPTMCM_GROUP_THREADS"] = "0"
    case(f"fuzz400 serial {what}", R, vol, spec, tf, spd, ld, params, mvp, layout, 6, 9)
    os.environ.pop("VPTMCM_GROUP_THREADS")
    vol2 = cf.fbm_volume(48, 35, nthreads=8)
    spd2, ld2 = np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32)
    p2 = dict(extinction=24.0, bounces=8, steps=8)
    for R2, n_rep in ((64, 3), (16, 3), (64, 2)):
        case("plain", R2, vol2, cf.spectrum_buffer("12"), cf.tf_spectral(), spd2, ld2, p2, cf.golden_mvp("orbit"),
             vptmcm.LAYOUT_COLUMN4, n_rep, 9)


if __name__ == "__main__":
    main()
