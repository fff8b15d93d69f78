"""Volume ingest readers: the JS BVPReader / ZIPReader / Volume
assemble a BVP archive's blocks at their placements exactly like
WebGPUVolume.readModality (WebGPUVolume.js:34-96) writes them into the texture."""
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

from bvp import write_bvp
from vptmcm import configs as cf

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")
@pytest.mark.parametrize("brick,deflate", [((32, 32, 32), 0), ((24, 40, 16), 3), ((64, 64, 1), 0)])
def test_bvp_archive_assembles_to_the_volume(tmp_path, brick, deflate):
    vol = cf.fbm_volume(64, 21)[:, :48, :56].copy()  # non-cubic, non-multiple-of-brick
    (tmp_path / "v.bvp").write_bytes(write_bvp(vol, brick, deflate))
    r = subprocess.run(["node", str(ROOT / "tests" / "js" / "bvp_read.js"), str(tmp_path / "v.bvp"),
                        str(tmp_path / "out.raw")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    meta = json.loads(r.stdout)
    assert (meta["width"], meta["height"], meta["depth"]) == (56, 48, 64)
    got = np.frombuffer((tmp_path / "out.raw").read_bytes(), np.uint8).reshape(vol.shape)
    assert np.array_equal(got, vol)
    nblocks = -(-56 // brick[0]) * -(-48 // brick[1]) * -(-64 // brick[2])
    assert meta["files"] == nblocks + 1
