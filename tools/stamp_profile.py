#!/usr/bin/env python3
"""Per-segment cycle breakdown of the march's volume steps (experiment build).

Runs the bench workload (C3) on build/variants/libvptmcm_<variant>.so built with
-DVPT_STAMP=1 (tools/variants.py stamp='-DVPT_STAMP=1'), settles the clock with
fused launches, then runs ONE one-pass launch whose waves write their
s_memtime segment sums into the fp32 image buffer (tile * 8 + k, see k_march).

    VPTMCM_LIB=stamp python tools/stamp_profile.py [--camera default] [--passes 4]

Prints one JSON line: per-volume-step cycles of each segment (median / mean
over the volume waves), the robust/all-exit step cost, and launch cycles.
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

SEG = ["head", "gather_issue_and_shadow", "gather_wait", "filter_tf_decision", "branches"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--camera", default="default")
    ap.add_argument("--layout", default="corner8")
    ap.add_argument("--volume", type=int, default=512)
    ap.add_argument("--samples", type=int, default=8, help="one-pass launches averaged")
    ap.add_argument("--tf", default="spectral", choices=["spectral", "materials", "materials_const"])
    ap.add_argument("--bins", default="12")
    ap.add_argument("--fused", type=int, default=32,
                    help="passes of a final fused launch whose clock is reported")
    ap.add_argument("--dump", default="", help="save the raw per-tile records (npz)")
    a = ap.parse_args()
    R, S = 512, 8
    layout = {"corner8": vptmcm.LAYOUT_CORNER8, "brick8": vptmcm.LAYOUT_BRICK8}[a.layout]
    r = vptmcm.Renderer(R, device=0, layout=layout)
    r.set_volume(cf.fbm_volume(a.volume, 512 if a.volume == 512 else a.volume))
    r.set_material_tf({"spectral": cf.tf_spectral, "materials": lambda: cf.tf_materials(True),
                       "materials_const": lambda: cf.tf_materials(False)}[a.tf]())
    spd, ldir = cf.light_default()
    r.set_light(spd, ldir)
    r.set_spectrum(cf.spectrum_buffer(a.bins))
    r.set_params(extinction=32.0, bounces=8, steps=S)
    mvp = cf.default_mvp_inverse() if a.camera == "default" else cf.golden_mvp(a.camera)
    seeds = cf.seed_stream(32, start=0)
    r.reset(mvp, seeds[0])
    for _ in range(300):  # ~150 ms of fused launches: clock settled
        r.render_passes(mvp, seeds[1:33])
    r.synchronize()
    acc = []
    for k in range(a.samples):
        r.render_passes(mvp, seeds[1 + k:2 + k])  # one-pass launch: 16-bit sums do not wrap
        r.synchronize()
        w = r.read_rgb().reshape(-1).view(np.uint32)[: (R * R // 64) * 8].reshape(-1, 8).copy()
        acc.append(w)
    # shader clock over a fused launch: s_memtime cycles / s_memrealtime (100 MHz)
    r.render_passes(mvp, seeds[1:1 + a.fused])
    r.synchronize()
    wf = r.read_rgb().reshape(-1).view(np.uint32)[: (R * R // 64) * 8].reshape(-1, 8).copy()
    r.close()
    if a.dump:
        np.savez_compressed(a.dump, fused=wf, **{f"one_pass_{k}": w for k, w in enumerate(acc)})
    live = wf[:, 6] > 0
    clk = wf[live, 4].astype(np.float64) / wf[live, 6] * 100.0  # MHz
    segs, walls, steps = [], [], []
    for w in acc:
        vol = ((w[:, 5] & 0xff) == 1) & (w[:, 3] > 0)
        lo = lambda x: (x & 0xFFFF).astype(np.float64)  # noqa: E731
        hi = lambda x: (x >> 16).astype(np.float64)  # noqa: E731
        n = (w[vol, 3] & 0xFFFF).astype(np.float64)
        seg = np.stack([lo(w[vol, 0]), hi(w[vol, 0]), lo(w[vol, 1]), hi(w[vol, 1]), lo(w[vol, 2])], 1)
        segs.append(seg / n[:, None])
        steps.append(n)
        walls.append(w[:, 4].astype(np.float64))
    seg = np.concatenate(segs)
    out = {"volume_waves": int(seg.shape[0] // a.samples), "camera": a.camera, "layout": a.layout,
           "tf": a.tf, "bins": a.bins,
           "volume": a.volume,
           "cycles_per_volume_step_median": {s: round(float(np.median(seg[:, i])), 1) for i, s in enumerate(SEG)},
           "cycles_per_volume_step_mean": {s: round(float(seg[:, i].mean()), 1) for i, s in enumerate(SEG)},
           "total_per_volume_step_median": round(float(np.median(seg.sum(1))), 1),
           "volume_steps_per_wave_median": float(np.median(np.concatenate(steps))),
           "launch_cycles_max": float(np.max(np.concatenate(walls))),
           "launch_cycles_median": float(np.median(np.concatenate(walls))),
           "clock_mhz_fused_launch_median": round(float(np.median(clk)), 1),
           "clock_mhz_one_pass": round(float(np.median(np.concatenate(
               [w[w[:, 6] > 0, 4] / w[w[:, 6] > 0, 6] * 100.0 for w in acc]))), 1),
           "fused_launch_us_max": round(float(wf[live, 6].max()) / 100.0, 2)}
    # where the volume waves of the fused launch ran: waves per SIMD (HW_ID:
    # SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC from hwreg 20)
    hw, xcc = wf[:, 7], (wf[:, 5] >> 8) & 0xff
    simd = (xcc.astype(np.int64) << 16) | (((hw >> 13) & 7) << 12) | (((hw >> 12) & 1) << 11) | \
        (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    volw = live & ((wf[:, 5] & 0xff) == 1)
    ids, cnt = np.unique(simd[volw], return_counts=True)
    out["distinct_simds_all_waves"] = int(len(np.unique(simd[live])))
    out["volume_waves_per_simd_hist"] = {int(k): int(v) for k, v in zip(*np.unique(cnt, return_counts=True))}
    dur = wf[:, 6].astype(np.float64) / 100.0  # us
    m = {}
    for k in sorted(set(cnt.tolist())):
        sel = np.isin(simd, ids[cnt == k]) & volw
        m[int(k)] = round(float(dur[sel].max()), 2)
    out["fused_volume_wave_us_max_by_simd_load"] = m
    # background waves by the volume-wave count of their SIMD
    load = dict(zip(ids.tolist(), cnt.tolist()))
    bgw = live & ((wf[:, 5] & 0xff) == 0)
    bl = np.array([load.get(int(x), 0) for x in simd])
    out["fused_background_wave_us_max_by_simd_load"] = {
        int(k): round(float(dur[bgw & (bl == k)].max()), 2) for k in sorted(set(bl[bgw].tolist()))}
    out["fused_background_wave_us_median_by_simd_load"] = {
        int(k): round(float(np.median(dur[bgw & (bl == k)])), 2) for k in sorted(set(bl[bgw].tolist()))}
    out["fused_volume_wave_us_median"] = round(float(np.median(dur[volw])), 2)
    sw, wd = (wf[:, 3] >> 16) & 0xFF, wf[:, 3] >> 24
    if sw.any() or wd.any():  # tile-swap builds: swaps / withdrawn offers / offer wait per wave
        out["swap"] = {"swaps_total": int(sw.sum()), "withdrawn_total": int(wd.sum()),
                       "waves_swapping": int((sw > 0).sum()),
                       "swaps_per_volume_wave_mean": round(float(sw[volw].mean()), 2),
                       "withdrawn_per_volume_wave_mean": round(float(wd[volw].mean()), 2)}
    # SIMDs holding two volume waves: when the first and the second of the pair end
    first, second = [], []
    for sid in ids[cnt == 2]:
        d = np.sort(dur[(simd == sid) & volw])
        first.append(d[0])
        second.append(d[-1])
    if first:
        out["fused_pair_wave_us_median"] = {"first": round(float(np.median(first)), 2),
                                            "second": round(float(np.median(second)), 2),
                                            "second_max": round(float(np.max(second)), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
