#!/usr/bin/env python3
"""Host-measured volume ingest time (block-wise ingest cost).

For each size: one set_volume (a single block), slice-by-slice ingest (1-slice
placements, as a RAW reader's placements arrive) and 64-slice blocks; each
ends with volume_end and a synchronize. Prints one JSON line per case.

    python tools/ingest_time.py [--sizes 512 1024] [--layout corner8]
"""
import argparse
import json
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
    ap.add_argument("--sizes", type=int, nargs="+", default=[512, 1024])
    ap.add_argument("--layout", choices=["corner8", "brick8"], default="corner8")
    a = ap.parse_args()
    layout = vptmcm.LAYOUT_CORNER8 if a.layout == "corner8" else vptmcm.LAYOUT_BRICK8
    r = vptmcm.Renderer(64, device=0, layout=layout)
    for n in a.sizes:
        vol = cf.fbm_volume(n, n)
        for case, slab in (("set_volume", n), ("slices_1", 1), ("blocks_64", 64)):
            best = None
            for _ in range(2):
                r.synchronize()
                t0 = time.perf_counter()
                if slab == n:
                    r.set_volume(vol)
                else:
                    r.volume_begin(vol.shape)
                    for z in range(0, n, slab):
                        r.volume_write_block((0, 0, z), vol[z:z + slab])
                    r.volume_end()
                r.synchronize()
                el = time.perf_counter() - t0
                best = el if best is None else min(best, el)
            print(json.dumps({"size": n, "layout": a.layout, "case": case, "blocks": -(-n // slab),
                              "ms": round(best * 1e3, 2),
                              "GB_per_s_host_bytes": round(vol.nbytes / best / 1e9, 2)}), flush=True)
        del vol
    r.close()


if __name__ == "__main__":
    main()
