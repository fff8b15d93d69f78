import sys, time, json
sys.path.insert(0, "vpt-spectral-volume-rendering_amd/python")
import vptmcm
t = time.perf_counter(); r = vptmcm.Renderer(512, device=0); r.close()
print(json.dumps({"first_single_ms": round((time.perf_counter() - t) * 1e3, 1)}))
for n in (1, 2, 4, 8):
    t = time.perf_counter(); g = vptmcm.Renderer(512, devices=[0] * n); dt = time.perf_counter() - t
    g.close()
    print(json.dumps({"n": n, "create_ms": round(dt * 1e3, 1)}))
