#!/usr/bin/env python3
"""Per-wave timeline of a cross-launch-balanced (carry) march launch against a
plain one (experiment build -DVPT_STAMP=2, never the product).

C3 at R = 512: L launches of 32 queued render() passes (the JS progressive
loop); the last launch's per-wave stamps are read back raw
(VPTMCM_CARRY_NOFINAL=1: no completion launch overwrites them, so the images
of this run are NOT the renderer's). Per wave: entry, pass loop done (µs from
the first entry), the tile's passes to do and done, owing, and its SIMD's
volume-wave count. Reports the loop-end times by class.

    VPTMCM_LIB=tl VPTMCM_CARRY_NOFINAL=1 VPTMCM_CARRY=1 python tools/carry_timeline.py
"""
import json
import os
import sys
import time
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
    return {"n": int(x.size), "min": round(float(x.min()), 1), "med": round(float(np.median(x)), 1),
            "p90": round(float(np.percentile(x, 90)), 1), "max": round(float(x.max()), 1)}


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    R = 512
    r = vptmcm.Renderer(R, device=0)
    r.set_volume(cf.fbm_volume(512, 512))
    r.set_material_tf(cf.tf_spectral())
    spd, ld = cf.light_default()
    r.set_light(spd, ld)
    r.set_spectrum(cf.spectrum_buffer("12"))
    r.set_params(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(32 * (L + 1) + 1, start=0)
    r.reset(mvp, seeds[0])
    t = time.perf_counter()
    ss = cf.seed_stream(32, start=1 << 20)
    while (time.perf_counter() - t) < 0.15:
        r.render_passes(mvp, ss)
        r.synchronize()
    k = 1
    for _ in range(L):
        for _ in range(32):
            r.render(mvp, seeds[k])
            k += 1
        owed = r.debug_owed()
    w = r.read_rgb().view(np.uint32).reshape(-1)[: (R // 8) ** 2 * 8].reshape(-1, 8)
    r.close()
    live = w[:, 0] != 0
    w = w[live]
    tt = w[:, :5].astype(np.int64)
    t0 = tt[:, 0].min()
    tt = ((tt - t0) & 0xFFFFFFFF).astype(np.float64) / 100.0
    vol = (w[:, 5] & 0xFF) == 1
    hw, xcc = w[:, 7], (w[:, 5] >> 8) & 0xFF
    simd = (xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) | \
        (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    extra = w[:, 6]
    todo, done, owing = extra >> 16, (extra >> 8) & 0xFF, extra & 1
    carry = bool((extra >> 16).any())
    # volume waves per SIMD: waves with passes to do whose tile entered the volume
    hot = vol & (todo > 0) if carry else vol
    ids, cnt = np.unique(simd[hot], return_counts=True)
    load = dict(zip(ids.tolist(), cnt.tolist()))
    nl = np.array([load.get(int(s), 0) for s in simd])
    end = tt[:, 3]
    out = {"carry": carry, "carry_bg": os.environ.get("VPTMCM_CARRY_BG", "0"), "launches": L, "waves": int(len(w)), "span_us": round(float(tt[:, 4].max()), 1),
           "owed_after": {"tiles": int((owed > 0).sum()), "total": int(owed.sum())}}
    if carry:
        stopped = hot & (done < todo)
        out["loop_end"] = {
            "lone_owing": q(end[hot & (nl == 1) & (owing == 1)]),
            "lone_not_owing": q(end[hot & (nl == 1) & (owing == 0)]),
            "paired_owing": q(end[hot & (nl == 2) & (owing == 1)]),
            "paired_not_owing_complete": q(end[hot & (nl == 2) & (owing == 0) & ~stopped]),
            "paired_stopped": q(end[hot & (nl >= 2) & stopped]),
            "lone_stopped": q(end[hot & (nl == 1) & stopped]),
            "background": q(end[~hot]),
            "background_beside_pairs": q(end[~hot & (nl >= 2)]),
            "background_beside_lone": q(end[~hot & (nl == 1)])}
        out["passes_done"] = {"lone": q(done[hot & (nl == 1)]), "paired": q(done[hot & (nl == 2)]),
                              "background_beside_pairs": q(done[~vol & (nl >= 2)]),
                              "background_beside_lone": q(done[~vol & (nl == 1)])}
        out["background_stopped"] = int((~vol & (todo > 0) & (done < todo)).sum())
        out["simd_load"] = {int(v): int((np.array(list(load.values())) == v).sum()) for v in set(load.values())}
    else:
        out["loop_end"] = {"lone": q(end[vol & (nl == 1)]), "paired": q(end[vol & (nl == 2)]),
                           "background": q(end[~vol]),
                           "background_beside_pairs": q(end[~vol & (nl >= 2)]),
                           "background_beside_lone": q(end[~vol & (nl == 1)])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
