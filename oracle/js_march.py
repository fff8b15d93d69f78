"""TEST INFRASTRUCTURE ONLY: Python driver of the JavaScript march re-execution
(oracle/mcm_march.js over worker_threads, oracle/js_baseline.js).

Used by tests/test_js_march.py (bit-exact against the C oracle) and by
bench.py's cpu_baseline leg (the north_star's scalar JS/CPU baseline).
"""
from __future__ import annotations

import json
import shutil
import subprocess
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent


def node() -> str | None:
    return shutil.which("node")


def _bits(a) -> list:
    return [int(v) for v in np.asarray(a, np.float32).ravel().view(np.uint32)]


def write_inputs(d: Path, R, vol, tf, light, light_dir, spectrum, mvp, seeds, *, extinction,
                 bounces=8, steps=8, blur=0.0) -> None:
    v = np.ascontiguousarray(vol, np.uint8)
    D, H, W = v.shape
    meta = {"R": int(R), "W": W, "H": H, "D": D, "mvp_bits": _bits(mvp),
            "inv_res_bits": _bits([1.0 / R, 1.0 / R]), "blur_bits": _bits([blur])[0],
            "extinction_bits": _bits([extinction])[0], "max_bounces": int(bounces),
            "steps": int(steps), "light_dir_bits": _bits(light_dir),
            "seeds": [int(s) for s in seeds]}
    (d / "meta.json").write_text(json.dumps(meta))
    v.tofile(d / "vol.bin")
    np.ascontiguousarray(tf, np.uint8).tofile(d / "tf.bin")
    np.ascontiguousarray(light, np.uint8).tofile(d / "light.bin")
    spec = np.zeros(64, np.float32)
    s = np.asarray(spectrum)
    spec[: s.size] = s.view(np.float32) if s.dtype == np.uint32 else s
    spec.tofile(d / "spec.bin")


def run_check(R, vol, tf, light, light_dir, spectrum, mvp, seeds, threads=4, **params):
    """Reset with seeds[0] and one pass per further seed; returns (photons u32
    [R*R, 36], rgb32 [R, R, 3], rgba16 [R, R, 4]) of the last pass."""
    with tempfile.TemporaryDirectory() as t:
        d = Path(t)
        write_inputs(d, R, vol, tf, light, light_dir, spectrum, mvp, seeds, **params)
        subprocess.run([node(), str(HERE / "js_baseline.js"), str(d), "check", str(threads)],
                       check=True, timeout=600)
        ph = np.fromfile(d / "photons.bin", np.uint32).reshape(R * R, 36)
        rgb = np.fromfile(d / "rgb32.bin", np.float32).reshape(R, R, 3)
        rgba = np.fromfile(d / "rgba16.bin", np.uint16).reshape(R, R, 4)
    return ph, rgb, rgba


def run_bench(R, vol, tf, light, light_dir, spectrum, mvp, seeds, threads, seconds, **params):
    """Passes over the whole R x R frame for `seconds`; returns node's JSON line."""
    with tempfile.TemporaryDirectory() as t:
        d = Path(t)
        write_inputs(d, R, vol, tf, light, light_dir, spectrum, mvp, seeds, **params)
        out = subprocess.run([node(), str(HERE / "js_baseline.js"), str(d), "bench", str(threads),
                              str(seconds)], check=True, capture_output=True, text=True,
                             timeout=seconds * 4 + 300)
    return json.loads(out.stdout.strip().splitlines()[-1])
