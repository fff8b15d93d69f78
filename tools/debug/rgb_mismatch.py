"""Debug helper: locate the first rgba16f mismatch of the C1 spectral ext=32 case
and print both sides plus a numpy fma re-evaluation of radiance_to_rgb."""
import sys
from pathlib import Path
REPO = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(REPO / "tests"), str(REPO / "oracle"), str(REPO / "vpt-spectral-volume-rendering_amd" / "python")]
import numpy as np
import oracle as orc
import vptmcm
from vptmcm import configs as cf
from pyref import fma32, F
from test_gpu_parity import make_pair

gpu, cpu = make_pair(64, cf.sphere_in_cube(64), cf.tf_spectral(), ext=32.0, layout=1)
mvp = cf.default_mvp_inverse()
seeds = cf.seed_stream(9, start=0)
gpu.reset(mvp, seeds[0]); cpu.reset(mvp, seeds[0])
spec = cf.spectrum_buffer("12")
for k, s in enumerate(seeds[1:], 1):
    gpu.render(mvp, s)
    rgb_c, want = cpu.render(mvp, s)
    got = gpu.read_rgba16f()
    if not np.array_equal(got, want):
        idx = np.argwhere(got != want)
        print("pass", k, "mismatch at", idx[:4])
        y, x, ch = idx[0]
        ph = gpu.read_photons()[y * 64 + x]
        print("photon words equal:", np.array_equal(ph, cpu.photons[y * 64 + x]))
        rad = ph[10:22].view(np.float32)
        print("rad", [float(v) for v in rad])
        nb = 12
        X = Y = Z = F(0)
        for i in range(nb):
            X = fma32(rad[i], spec[2 + nb + i], X); Y = fma32(rad[i], spec[2 + 2 * nb + i], Y); Z = fma32(rad[i], spec[2 + 3 * nb + i], Z)
        r = fma32(F(-0.498536), Z, fma32(F(-1.537150), Y, F(3.240479) * X))
        g = fma32(F(0.041556), Z, fma32(F(1.875990), Y, F(-0.969255) * X))
        b = fma32(F(1.057311), Z, fma32(F(-0.204041), Y, F(0.055647) * X))
        print("XYZ", X, Y, Z, "pyref rgb", r, g, b, "oracle rgb32", rgb_c[y, x])
        print("gpu half", got[y, x], got[y, x].view(np.float16), "oracle half", want[y, x], want[y, x].view(np.float16))
        print("np f16 of pyref", np.float16(r), np.float16(g), np.float16(b))
        break
