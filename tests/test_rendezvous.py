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


def test_stale_payload_of_another_attempt_is_ignored(monkeypatch):
    """A file left by a crashed attempt (another restart count) under the same
    path is not taken: the payload must name the reader's own job key."""
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    key = rendezvous.job_key()
    path = rendezvous.uid_path(key)
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    stale_key = rendezvous.job_key()
    assert stale_key != key
    path.write_bytes(rendezvous._payload(stale_key, bytes(128)))  # wrong key inside
    try:
        import pytest
        with pytest.raises(TimeoutError):
            rendezvous.exchange_unique_id(1, None, key=key, timeout_s=0.2)
        # rank 0 of the new attempt replaces it; rank 1 then reads the new id
        rendezvous.exchange_unique_id(0, lambda: bytes(range(128)), key=key)
        assert rendezvous.exchange_unique_id(1, None, key=key, timeout_s=5) == bytes(range(128))
    finally:
        rendezvous.cleanup(key)


def _join_worker(rank, world, key, q, done):
    rendezvous.join(rank, world, key=key, timeout_s=30)
    q.put(rank)
    done.wait(60)  # a rank stays alive past the join (a marker counts only while its process runs)


def test_join_all_ranks_present():
    key = f"join-{os.getpid()}"
    ctx = mp.get_context("spawn")
    q, done = ctx.Queue(), ctx.Event()
    procs = [ctx.Process(target=_join_worker, args=(r, 3, key, q, done)) for r in (2, 0, 1)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=60) for _ in procs)
    done.set()
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert got == [0, 1, 2]
    rendezvous.cleanup(key, 3)
    assert not any(rendezvous.join_path(key, r).exists() for r in range(3))


def test_join_missing_rank_is_ecomm():
    """Rank 1 never arrives: rank 0 fails in the rendezvous, bounded, with the
    communicator error code, naming the missing rank."""
    import time

    import pytest
    import vptmcm
    key = f"join-missing-{os.getpid()}"
    t0 = time.monotonic()
    with pytest.raises(rendezvous.RendezvousError) as ei:
        rendezvous.join(0, 2, key=key, timeout_s=0.5)
    assert 0.5 <= time.monotonic() - t0 < 10
    assert ei.value.code == vptmcm.ECOMM and isinstance(ei.value, vptmcm.VptError)
    assert "[1]" in str(ei.value)
    rendezvous.cleanup(key, 2)


def test_join_timeout_from_environment(monkeypatch):
    monkeypatch.setenv("VPTMCM_COMM_TIMEOUT_MS", "2500")
    assert rendezvous.default_timeout_s() == 2.5
    monkeypatch.setenv("VPTMCM_COMM_TIMEOUT_MS", "junk")
    assert rendezvous.default_timeout_s() == 120.0


def test_stale_join_marker_is_not_a_live_peer(tmp_path):
    """A join marker left by a rank that is gone (a crashed job with the same
    key, or a reused pid with another start time) does not count as present:
    rank 0 still fails in the rendezvous, and removes its own marker when it
    does."""
    import subprocess
    import sys

    import pytest
    key = f"stale-{os.getpid()}"
    p = subprocess.run([sys.executable, "-c", "import os; print(os.getpid())"], capture_output=True,
                       text=True, check=True)
    dead = int(p.stdout)
    rendezvous.join_path(key, 1).write_text(f"{key}\n{dead}\n12345")  # a rank that exited
    rendezvous.join_path(key, 2).write_text(f"{key}\n{os.getpid()}\n1")  # live pid, wrong start time
    try:
        assert not rendezvous.marker_alive(rendezvous.join_path(key, 1), key)
        assert not rendezvous.marker_alive(rendezvous.join_path(key, 2), key)
        with pytest.raises(rendezvous.RendezvousError, match=r"\[1, 2\]"):
            rendezvous.join(0, 3, key=key, timeout_s=0.3)
        assert not rendezvous.join_path(key, 0).exists()  # its own marker is gone
        # a live marker of the same key from this very process counts
        rendezvous.join(0, 1, key=key, timeout_s=5)
        assert rendezvous.marker_alive(rendezvous.join_path(key, 0), key)
    finally:
        rendezvous.cleanup(key, 3)
