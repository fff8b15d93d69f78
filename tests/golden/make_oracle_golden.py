"""Writes tests/golden/oracle_regression.json: a hash of the oracle's own output
for a fixed case, so any change to the arithmetic specification is deliberate.
Run: python tests/golden/make_oracle_golden.py"""
import hashlib
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parent), str(HERE.parents[1] / "oracle"),
                str(HERE.parents[1] / "vpt-spectral-volume-rendering_amd" / "python")]
import oracle as orc  # noqa: E402
from vptmcm import configs as cf  # noqa: E402

R = 32
o = orc.Oracle(R)
o.set_spectrum(cf.spectrum_buffer("12"))
o.volume, o.tf, o.light = cf.sphere_in_cube(64), cf.tf_spectral(), cf.light_default()[0]
o.params.update(extinction=32.0)
mvp = cf.default_mvp_inverse()
seeds = cf.seed_stream(3, start=0)
o.reset(mvp, seeds[0])
for s in seeds[1:]:
    _, rgba = o.render(mvp, s)
h = hashlib.sha256(o.photons.tobytes() + rgba.tobytes()).hexdigest()
(HERE / "oracle_regression.json").write_text(json.dumps(
    {"sha256_R32_sphere64_tf3_ext32_2pass": h}, indent=1) + "\n")
print(h)
