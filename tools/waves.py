#!/usr/bin/env python3
"""Analyse per-wave records (VPTMCM_WAVE_DUMP from the experiment build)."""
import sys
import numpy as np

def load(path, n):
    r = np.fromfile(path, np.uint32).reshape(-1, 8)[:n]
    hw = r[:, 0]
    d = dict(wave=hw & 0xF, simd=(hw >> 4) & 3, cu=(hw >> 8) & 0xF, sh=(hw >> 12) & 1,
             se=(hw >> 13) & 7, xcc=r[:, 1] & 0xF, rt0=r[:, 2].astype(np.int64), rt1=r[:, 3].astype(np.int64),
             cyc=r[:, 4], tile=r[:, 5], ent=r[:, 6], bw=r[:, 7])
    t0 = d["rt0"].min()
    d["rt0"] -= t0
    d["rt1"] -= t0
    return d

for path in sys.argv[1:]:
    d = load(path, 4096)
    w = d["bw"] % 16
    print(path)
    print("  SIMD vs w%4 agreement", np.mean(d["simd"] == w % 4), " vs w//4", np.mean(d["simd"] == w // 4))
    print("  start spread (10ns ticks): min %d max %d" % (d["rt0"].min(), d["rt0"].max()),
          " end: median %d max %d" % (np.median(d["rt1"]), d["rt1"].max()))
    for e in (0, 1):
        m = d["ent"] == e
        print("  entered=%d waves %d  cycles mean %.0f max %.0f  dur(ticks) mean %.0f max %.0f" % (
            e, m.sum(), d["cyc"][m].mean(), d["cyc"][m].max(), (d["rt1"] - d["rt0"])[m].mean(),
            (d["rt1"] - d["rt0"])[m].max()))
    key = d["xcc"] * 4096 + d["se"] * 512 + d["sh"] * 256 + d["cu"] * 16 + d["simd"]
    u, inv = np.unique(key, return_inverse=True)
    nvol = np.bincount(inv, weights=d["ent"])
    print("  distinct SIMDs", len(u), " volume waves per SIMD histogram", np.bincount(nvol.astype(int)))
    end = np.zeros(len(u)); np.maximum.at(end, inv, d["rt1"])
    for k in range(int(nvol.max()) + 1):
        if (nvol == k).any():
            print("    SIMDs with %d volume waves: last end mean %.0f max %.0f" % (k, end[nvol == k].mean(), end[nvol == k].max()))
