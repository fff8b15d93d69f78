#!/usr/bin/env python3
"""Bit-identity of two builds of the library on the benchmark workload (analysis).

    VPTMCM_LIB=<variant> python tools/ab_bits.py dump out.json [--passes 64] [--fuse 32]
    python tools/ab_bits.py cmp a.json b.json

`dump` runs C3 (512^3 fBm, R = 512, S = 8) from a reset through `passes` passes in
fused launches and writes SHA-256 digests of the photon words, the fp32 image and
the rgba16f image; `cmp` requires the two digests to match (bit for bit) (timing-only variants
such as the tile swap must not change a single bit).
"""
import argparse
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]


def dump(a):
    import vptmcm
    from vptmcm import configs as cf
    r = vptmcm.Renderer(a.resolution, device=0)
    r.set_volume(cf.fbm_volume(a.volume, 512 if a.volume == 512 else a.volume))
    r.set_material_tf(cf.tf_materials(True) if a.tf == "materials" else cf.tf_spectral())
    r.set_light(*cf.light_default())
    r.set_spectrum(cf.spectrum_buffer(a.bins))
    r.set_params(extinction=32.0, bounces=8, steps=8)
    mvp = cf.default_mvp_inverse()
    seeds = cf.seed_stream(a.passes + 1, start=0)
    r.reset(mvp, seeds[0])
    done = 0
    while done < a.passes:
        n = min(a.fuse, a.passes - done)
        r.render_passes(mvp, seeds[1 + done:1 + done + n])
        done += n
    import hashlib
    import json
    out = {k: hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()
           for k, v in (("photons", r.read_photons()), ("rgb", r.read_rgb()), ("rgba", r.read_rgba16f()))}
    out["launch"] = r.last_launch()
    Path(a.out).write_text(json.dumps(out))
    r.close()


def cmp(a):
    import json
    x, y = json.loads(Path(a.a).read_text()), json.loads(Path(a.b).read_text())
    same = {k: x[k] == y[k] for k in ("photons", "rgb", "rgba")}
    print(json.dumps({"identical": same, "launch_a": x["launch"], "launch_b": y["launch"]}))
    sys.exit(0 if all(same.values()) else 1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("dump")
    d.add_argument("out")
    d.add_argument("--passes", type=int, default=64)
    d.add_argument("--fuse", type=int, default=32)
    d.add_argument("--resolution", type=int, default=512)
    d.add_argument("--volume", type=int, default=512)
    d.add_argument("--tf", default="spectral", choices=["spectral", "materials"])
    d.add_argument("--bins", default="12")
    c = sub.add_parser("cmp")
    c.add_argument("a")
    c.add_argument("b")
    a = ap.parse_args()
    dump(a) if a.cmd == "dump" else cmp(a)
