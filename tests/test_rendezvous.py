"""Torch-free unique-id exchange used to bootstrap RCCL (2 processes, CPU)."""
import multiprocessing as mp
import os

from vptmcm import rendezvous


def _worker(rank, key, q):
    uid = rendezvous.exchange_unique_id(rank, lambda: bytes(range(128)), key=key, timeout_s=30)
    q.put((rank, uid))


def test_two_process_exchange():
    key = f"test-{os.getpid()}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, key, q)) for r in (1, 0)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    rendezvous.cleanup(key)
    assert out[0] == out[1] == bytes(range(128))
    assert not rendezvous.uid_path(key).exists()


def test_env_world_defaults(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert rendezvous.env_world() == (0, 1, 0)
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert rendezvous.env_world() == (3, 4, 3)
