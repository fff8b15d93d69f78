#!/usr/bin/env python3
"""Two RCCL ranks on ONE GPU (measurement aid; does RCCL accept a repeated
device?). If it does, the N = 2 composite paths run for real on a one-GPU box:
each rank renders its own seed stream, then the all-reduce and the sharded
reduce-scatter (+ all-gather at read) composites are compared with the host
sum of both ranks' k_pack buffers. One JSON line per rank; exit 0 when both
agree (or a clean "rccl refused" record when RCCL rejects the layout).

    python tools/rccl_two_ranks_one_gpu.py
"""
import json
import multiprocessing as mp
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "vpt-spectral-volume-rendering_amd" / "python"))


def rank_main(rank: int, uq, q):
    import numpy as np
    import vptmcm
    from vptmcm import configs as cf
    out = {"rank": rank}
    try:
        # rank 0 makes the unique id and hands it on (the parent never touches the GPU)
        if rank == 0:
            uid = vptmcm.unique_id()
            uq.put(uid)
        else:
            uid = uq.get(timeout=120)
        R = 64
        g = vptmcm.Renderer(R, device=0)
        g.set_spectrum(cf.spectrum_buffer("12"))
        g.set_volume(cf.fbm_volume(48, 21, nthreads=4))
        g.set_material_tf(cf.tf_spectral())
        g.set_light(np.full(256, 100, np.uint8), np.asarray((1, 0, 0), np.float32))
        g.set_params(extinction=24.0, bounces=8, steps=8)
        t0 = time.time()
        g.comm_init(uid, 2, rank)
        out["comm_init_s"] = round(time.time() - t0, 2)
        mvp = cf.default_mvp_inverse()
        seeds = cf.seed_stream(12, start=7, rank=rank)
        g.reset(mvp, seeds[0])
        res = {}
        for k, (inline, sharded) in enumerate([(False, False), (True, True), (False, True)]):
            g.render_passes(mvp, seeds[1 + 3 * k: 4 + 3 * k])
            pk = g.pack_radiance()
            g.allreduce_radiance(inline=inline, sharded=sharded)
            rgb, n = g.read_composite()
            res[f"{inline}-{sharded}"] = (pk, rgb, n)
        q.put((rank, {key: (v[0].tolist(), v[1].tolist(), v[2].tolist()) for key, v in res.items()}))
        g.barrier()
        g.close()
        out["ok"] = True
    except Exception as e:  # a refused layout is a result, not a crash
        out["ok"] = False
        out["error"] = repr(e)[:400]
        q.put((rank, None))
    print(json.dumps(out), flush=True)


def main():
    import numpy as np
    ctx = mp.get_context("spawn")
    q, uq = ctx.Queue(), ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, uq, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(2):
        r, v = q.get(timeout=240)
        got[r] = v
    for p in ps:
        p.join(timeout=60)
    if any(v is None for v in got.values()):
        print(json.dumps({"result": "rccl refused or failed"}))
        return 0
    report = {}
    for key in got[0]:
        pk = [np.asarray(got[r][key][0], np.float32) for r in range(2)]
        s = pk[0] + pk[1]  # both terms of a 2-rank sum: the order does not matter
        with np.errstate(divide="ignore", invalid="ignore"):
            want = np.where(s[..., 3:] > 0, s[..., :3] / s[..., 3:], np.float32(0)).astype(np.float32)
        same = [np.array_equal(np.asarray(got[r][key][1], np.float32), want) for r in range(2)]
        cnt = [np.array_equal(np.asarray(got[r][key][2], np.float32), s[..., 3]) for r in range(2)]
        report[key] = {"rgb_bitexact": same, "counts": cnt}
    print(json.dumps({"result": report}))
    return 0 if all(all(v["rgb_bitexact"]) and all(v["counts"]) for v in report.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
