"""World-size-2 gloo test of the photon-parallel composite (CPU).

Each rank renders its own replica of the frame with its rank seed stream
(configs.seed_bits(k, rank); rank 0 == the 1-GPU stream) using the CPU oracle,
packs (rgb*n, n) per pixel exactly as k_pack does (rgb = the last pass's fp32
radiance_to_rgb image, read_rgb; n = photon sample count; f32 products),
all-reduces over gloo and checks the composite against the single-process sum
of both replicas.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

R = 16


def _replica(rank):
    import oracle as orc
    from vptmcm import configs as cf
    o = orc.Oracle(R)
    o.set_spectrum(cf.spectrum_buffer("12"))
    o.volume, o.tf, o.light = cf.sphere_in_cube(32), cf.tf_spectral(), cf.light_default()[0]
    o.params.update(extinction=8.0)
    mvp = cf.default_mvp_inverse()
    o.reset(mvp, cf.seed_bits(0, rank), nthreads=1)
    for k in range(1, 4):
        rgb, _ = o.render(mvp, cf.seed_bits(k, rank), nthreads=1)
    n = o.photons[:, 7].astype(np.float32).reshape(R, R)
    rgb = np.asarray(rgb, np.float32).reshape(R, R, 3)
    return np.concatenate([rgb * n[..., None], n[..., None]], axis=-1).astype(np.float32)


def _run(rank, world, port, out):
    import sys
    sys.path[:0] = out["paths"]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    packed = torch.from_numpy(_replica(rank))
    dist.all_reduce(packed)
    if rank == 0:
        np.save(out["file"], packed.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_composite_two_ranks(tmp_path):
    import sys
    f = tmp_path / "comp.npy"
    port = 29500 + os.getpid() % 1000
    tmp.spawn(_run, args=(2, port, {"paths": sys.path[:6], "file": str(f)}), nprocs=2, join=True)
    got = np.load(f)
    want = _replica(0) + _replica(1)
    np.testing.assert_array_equal(got, want)
    rgb = got[..., :3] / got[..., 3:]
    assert np.isfinite(rgb).all() and (got[..., 3] >= 1).all()
    # rank 0's replica is the single-GPU run (same seed stream)
    assert not np.array_equal(_replica(0), _replica(1))
