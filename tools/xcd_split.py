#!/usr/bin/env python3
"""Per-XCD view of a launch timeline dump (tools/timeline_profile.py --dump):
for every XCD, the SIMDs that hold two volume waves (pairs) and one, and when
their volume waves end (µs from the launch's first wave entry).

    python tools/xcd_split.py raw.npz [F32_0 ...]   -> one JSON line per launch
"""
import json
import sys

import numpy as np


def split(w):
    t = w[:, :5].astype(np.int64)
    t = ((t - t[:, 0].min()) & 0xFFFFFFFF) / 100.0
    vol = (w[:, 5] & 0xFF) == 1
    hw, xcc = w[:, 7], (w[:, 5] >> 8) & 0xFF
    simd = (xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) | \
        (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    ids, cnt = np.unique(simd[vol], return_counts=True)
    out = {"span_us": round(float(t[:, 4].max()), 2), "xcd": {}}
    for x in range(8):
        row = {}
        for name, k in (("pairs", 2), ("lone", 1)):
            m = np.isin(simd, ids[cnt == k]) & vol & (xcc == x)
            row[name] = int(m.sum() // k)
            if m.any():
                row[name + "_end_med"] = round(float(np.median(t[m, 4])), 1)
                row[name + "_end_max"] = round(float(t[m, 4].max()), 1)
        out["xcd"][x] = row
    return out


if __name__ == "__main__":
    z = np.load(sys.argv[1])
    for key in sys.argv[2:] or sorted(k for k in z.files if k.endswith("_0")):
        print(json.dumps({"launch": key, **split(z[key])}))
