"""Writes BVP volume archives for the reader tests: a zip with manifest.json
(modalities / placements / blocks, the structure WebGPUVolume.readModality and
BVPReader consume, WebGPUVolume.js:34-96, BVPReader.js:13-29) and one raw u8
file per block. Test helper only."""
import io
import json
import zipfile

import numpy as np


def write_bvp(vol: np.ndarray, brick=(32, 32, 32), deflate_every=0) -> bytes:
    """vol is [D, H, W] u8; bricks are (bw, bh, bd); every `deflate_every`-th
    block is stored deflated (0 = all stored, as the reference's tools write)."""
    D, H, W = vol.shape
    bw, bh, bd = brick
    blocks, placements, files = [], [], []
    for z in range(0, D, bd):
        for y in range(0, H, bh):
            for x in range(0, W, bw):
                b = np.ascontiguousarray(vol[z:z + bd, y:y + bh, x:x + bw])
                i = len(blocks)
                url = f"blocks/block-{i}.raw"
                blocks.append({"url": url, "format": "raw",
                               "dimensions": {"width": b.shape[2], "height": b.shape[1], "depth": b.shape[0]}})
                placements.append({"index": i, "position": {"x": x, "y": y, "z": z}})
                files.append((url, b.tobytes()))
    manifest = {"meta": {"version": 1},
                "modalities": [{"name": "default", "dimensions": {"width": W, "height": H, "depth": D},
                                "transform": {"matrix": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]},
                                "format": "r8unorm", "placements": placements}],
                "blocks": blocks}
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr(zipfile.ZipInfo("manifest.json"), json.dumps(manifest))
        for k, (url, data) in enumerate(files):
            zi = zipfile.ZipInfo(url)
            zi.compress_type = zipfile.ZIP_DEFLATED if deflate_every and k % deflate_every == 0 \
                else zipfile.ZIP_STORED
            z.writestr(zi, data)
    return buf.getvalue()
