#!/usr/bin/env python3
"""Render a PNG through the drop-in JS host (tools/render_png.js): C3's fBm
volume (at --volume^3), spectral TF, 12 bins, extinction 32, default camera,
--passes progressive passes, then the artistic tone mapper (analysis / demo).

    python tools/render_png.py out.png [--resolution 512] [--volume 512] [--passes 256]
"""
import argparse
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
from vptmcm import configs as cf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--resolution", type=int, default=512)
    ap.add_argument("--volume", type=int, default=512)
    ap.add_argument("--passes", type=int, default=256)
    ap.add_argument("--tf", default="spectral", choices=["spectral", "materials"])
    a = ap.parse_args()
    vol = cf.fbm_volume(a.volume, 512 if a.volume == 512 else a.volume)
    tf = cf.tf_spectral() if a.tf == "spectral" else cf.tf_materials(True)
    with tempfile.TemporaryDirectory(prefix="vptmcm-png-") as d:
        d = Path(d)
        vol.tofile(d / "vol.raw")
        np.ascontiguousarray(tf, np.uint8).tofile(d / "tf.bin")
        np.ascontiguousarray(cf.spectrum_buffer("12"), np.float32).tofile(d / "spec.bin")
        D, H, W = vol.shape
        case = dict(R=a.resolution, W=W, H=H, D=D, volume_path=str(d / "vol.raw"),
                    tf_path=str(d / "tf.bin"), spectrum_path=str(d / "spec.bin"), extinction=32.0,
                    passes=a.passes, gamma=2.2)
        (d / "case.json").write_text(json.dumps(case))
        r = subprocess.run(["node", str(REPO / "tools" / "render_png.js"), str(d / "case.json"),
                            str(Path(a.out).resolve())], capture_output=True, text=True, timeout=600)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
