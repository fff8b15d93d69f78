#!/usr/bin/env python3
"""Doubly loaded SIMDs per XCD under the XCD-speed-aware deal (variant bit 8):
C3, 32-pass launches; after 1, 10, 50, 100, 300 and 600 launches the deal of
the last launch (vptmcm_debug_schedule) gives volume tiles per XCD (blocks
b with b % 8 == x) minus the 128 SIMDs each XCD holds once.

    VPTMCM_MARCH_VARIANT=256 python tools/xcd_quota_probe.py
"""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
import vptmcm  # noqa: E402
from vptmcm import configs as cf  # noqa: E402

r = vptmcm.Renderer(512, device=0)
r.set_volume(cf.fbm_volume(512, 512))
r.set_material_tf(cf.tf_spectral())
spd, ldir = cf.light_default()
r.set_light(spd, ldir)
r.set_spectrum(cf.spectrum_buffer("12"))
r.set_params(extinction=32.0, bounces=8, steps=8)
mvp = cf.default_mvp_inverse()
seeds = cf.seed_stream(33, start=0)
r.reset(mvp, seeds[0])
done, out = 0, {}
for mark in (1, 10, 50, 100, 300, 600):
    while done < mark:
        r.render_passes(mvp, seeds[1:33])
        done += 1
    tab = r.debug_schedule()
    G = tab.size // 16
    vol = ((tab != 0xFFFFFFFF) & ((tab >> 31) == 1)).reshape(G, 16).sum(1)
    per_xcd = [int(vol[x::8].sum()) - 4 * (G // 8) for x in range(8)]
    out[mark] = per_xcd
r.close()
print(json.dumps({"pairs_per_xcd_after_launches": out}))
