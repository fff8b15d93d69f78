#!/usr/bin/env python3
"""Times the JavaScript march re-execution (oracle/js_baseline.js) on the bench
workload outside bench.py (measurement aid). Usage: tools/js_baseline_time.py [threads] [seconds]"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "oracle"), str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
import js_march  # noqa: E402
from vptmcm import configs as cf  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
t = time.time()
vol = cf.fbm_volume(512, 512)
print("volume", round(time.time() - t, 2), "s")
spd, ld = cf.light_default()
print(js_march.run_bench(512, vol, cf.tf_spectral(), spd, ld, cf.spectrum_buffer("12"),
                         cf.default_mvp_inverse(), cf.seed_stream(40, start=0), threads=threads,
                         seconds=seconds, extinction=32.0))
