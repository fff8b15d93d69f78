#!/usr/bin/env python3
"""Wave-level branch statistics of the march on the bench workload (analysis tool).

Runs the C oracle (built with tools/march_stats.c's outcome hook) over a few
passes of BASELINE C3 and reports, per photon-step and per 64-lane 8x8 tile-step,
how often the four outcomes occur — the numbers that decide what a wave pays
for the divergent reset / scatter paths. Usage: python tools/march_stats.py [R] [passes]
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python"), str(REPO / "oracle")]
from vptmcm import configs as cf  # noqa: E402
import oracle as orc  # noqa: E402

OUT = Path("/tmp/march_stats")


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    S = 8
    OUT.mkdir(exist_ok=True)
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-std=c11", "-D_GNU_SOURCE", "-ffp-contract=off",
                    str(REPO / "tools/march_stats.c"), f"-I{REPO / 'oracle'}", "-o",
                    str(OUT / "liboracle.so"), "-lm", "-lpthread"], check=True)
    orc.HERE, orc._L = OUT, None
    L = orc.load()
    ev = np.zeros((R, R, S), np.uint8)
    L.stats_set_buffer(C.c_void_p(ev.ctypes.data), R, S)
    vol = cf.fbm_volume(512, 512)
    o = orc.Oracle(R)
    o.set_spectrum(cf.spectrum_buffer("12"))
    o.volume, o.tf = vol, cf.tf_spectral()
    o.light, o.light_dir = cf.light_default()
    o.params.update(extinction=32.0, bounces=8, steps=S)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(passes + 1, start=0)
    o.reset(mvp, seeds[0])
    tot = np.zeros(4)
    wave = {k: 0 for k in ("steps", "any_term", "any_exit", "any_abs", "any_scat", "all_null",
                           "all_exit", "some_inside", "inside_any_term", "inside_any_scat",
                           "inside_all_null", "inside_null_lanes", "inside_lanes")}
    for k in range(passes):
        o.render(mvp, seeds[1 + k])
        if k == 0:
            continue  # first pass after reset: skip
        tot += np.bincount(ev.ravel(), minlength=4)
        t = ev.reshape(R // 8, 8, R // 8, 8, S).transpose(0, 2, 1, 3, 4).reshape(-1, 64, S)
        term = (t >= 2).any(1)
        ex = (t == 3)
        inside = ~ex.all(1)
        wave["steps"] += term.size
        wave["any_term"] += term.sum()
        wave["any_exit"] += ex.any(1).sum()
        wave["any_abs"] += (t == 2).any(1).sum()
        wave["any_scat"] += (t == 1).any(1).sum()
        wave["all_null"] += (t == 0).all(1).sum()
        wave["all_exit"] += ex.all(1).sum()
        wave["some_inside"] += inside.sum()
        wave["inside_any_term"] += (term & inside).sum()
        wave["inside_any_scat"] += ((t == 1).any(1) & inside).sum()
        wave["inside_all_null"] += ((t == 0).all(1) & inside).sum()
        wave["inside_null_lanes"] += ((t == 0).sum(1) * inside).sum()
        wave["inside_lanes"] += 64 * inside.sum()
    n = tot.sum()
    print(f"photon-steps: null {tot[0]/n:.3f} scatter {tot[1]/n:.3f} absorb {tot[2]/n:.3f} exit {tot[3]/n:.3f}")
    ws = wave["steps"]
    for k, v in wave.items():
        if k not in ("steps",):
            print(f"  {k}: {v / ws:.3f}" if not k.startswith("inside_") else
                  f"  {k}: {v / max(1, wave['some_inside']):.3f}")
    print(f"  null lanes among inside wave-steps: {wave['inside_null_lanes']/max(1,wave['inside_lanes']):.3f}")


if __name__ == "__main__":
    main()
