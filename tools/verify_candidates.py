import sys, json
sys.path.insert(0, '/root/repo/vpt-spectral-volume-rendering_amd/python')
import vptmcm
res = {}
with vptmcm.Renderer(8, device=0) as g:
    for fn in (18, 19):
        bad, first = g.debug_verify(fn, 0, 1 << 32, 16)
        # restricted: positive normals with biased exponent 32..254 (sqrt_cr's proven range)
        lo, hi = 32 << 23, 255 << 23
        bad_r, first_r = g.debug_verify(fn, lo, hi - lo, 16)
        res[fn] = {"all": int(bad), "first": [hex(int(v)) for v in first[:8]],
                   "exp32_254": int(bad_r), "first_r": [hex(int(v)) for v in first_r[:8]]}
print(json.dumps(res))
