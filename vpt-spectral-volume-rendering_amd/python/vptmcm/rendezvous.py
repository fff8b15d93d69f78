"""Torch-free bootstrap of the RCCL communicator for one-process-per-GPU runs.

Under `torch.distributed.run` every local rank is a child of the same elastic
agent, so (parent pid, MASTER_PORT, run id) names the job uniquely on the
node. Every rank first publishes a join marker and waits, bounded, until all
ranks have (join: no rank enters RCCL's bootstrap while a peer is missing).
Rank 0 then publishes the 128-byte ncclUniqueId through an atomically
renamed file in the temp dir; the other ranks poll for it. Everything after
that (barriers, max-over-ranks timing) runs over RCCL itself, so the
benchmark never loads a second HIP runtime (torch's) into the process.
Single node only, which is all the benchmark uses.
"""
from __future__ import annotations

import atexit
import os
import tempfile
import time
from pathlib import Path

from ._lib import ECOMM, VptError


def env_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def job_key() -> str:
    """(agent pid, MASTER_PORT, run id, restart count): unique per elastic attempt,
    so a restarted job never reads an id a crashed attempt left behind."""
    parts = [str(os.getppid()), os.environ.get("MASTER_PORT", "0"),
             os.environ.get("TORCHELASTIC_RUN_ID", "none"),
             os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")]
    return "-".join(p.replace("/", "_") for p in parts)


def uid_path(key: str) -> Path:
    return Path(tempfile.gettempdir()) / f"vptmcm-uid-{key}.bin"


_MAGIC = b"VPTMCMUID1"


def _payload(key: str, uid: bytes) -> bytes:
    k = key.encode()
    return _MAGIC + len(k).to_bytes(2, "little") + k + uid


def _parse(key: str, data: bytes) -> bytes | None:
    """The uid if data is a complete payload published for exactly this key."""
    k = key.encode()
    head = _MAGIC + len(k).to_bytes(2, "little") + k
    if data.startswith(head) and len(data) == len(head) + 128:
        return data[len(head):]
    return None


def exchange_unique_id(rank: int, make_uid, key: str | None = None,
                       timeout_s: float = 180.0) -> bytes:
    """Rank 0 calls make_uid() and publishes it; others wait for a payload that
    names their own job key (a stale file of another attempt is ignored)."""
    key = key or job_key()
    path = uid_path(key)
    if rank == 0:
        uid = make_uid()
        assert len(uid) == 128
        try:
            path.unlink()  # whatever an earlier crashed attempt left
        except FileNotFoundError:
            pass
        tmp = path.with_name(path.name + f".{os.getpid()}.tmp")
        tmp.write_bytes(_payload(key, uid))
        os.replace(tmp, path)
        return uid
    deadline = time.monotonic() + timeout_s
    while time.monotonic() < deadline:
        try:
            uid = _parse(key, path.read_bytes())
            if uid is not None:
                return uid
        except FileNotFoundError:
            pass
        time.sleep(0.02)
    raise TimeoutError(f"rank {rank}: no unique id at {path} after {timeout_s}s")


class RendezvousError(VptError):
    """A peer rank never reached the rendezvous: raised before any RCCL call,
    with the communicator error code (ECOMM), so callers handle it like a
    failed communicator."""

    def __init__(self, msg: str):
        super().__init__(ECOMM, msg)


def join_path(key: str, rank: int) -> Path:
    return Path(tempfile.gettempdir()) / f"vptmcm-join-{key}-{rank}"


def default_timeout_s() -> float:
    """VPTMCM_COMM_TIMEOUT_MS (the library's communicator bound), default 120 s."""
    try:
        ms = int(os.environ.get("VPTMCM_COMM_TIMEOUT_MS", "120000"))
    except ValueError:
        ms = 120000
    return (ms if ms > 0 else 120000) / 1e3


def _proc_start(pid: int) -> str | None:
    """The process's start time in clock ticks since boot (/proc/<pid>/stat
    field 22), or None if no such process: with the pid it names one process
    for the boot's lifetime, whatever pids the kernel reuses."""
    try:
        stat = Path(f"/proc/{pid}/stat").read_text()
    except OSError:
        return None
    return stat[stat.rindex(")") + 2:].split()[19]


def _marker(key: str) -> bytes:
    pid = os.getpid()
    return f"{key}\n{pid}\n{_proc_start(pid)}".encode()


def marker_alive(path: Path, key: str) -> bool:
    """A join marker of this job key whose writer is still running (same pid
    and start time): a marker left by a rank that timed out or crashed, or by
    an earlier job with the same key, does not count as a live peer."""
    try:
        k, pid, start = path.read_text().split("\n")
    except (OSError, ValueError):
        return False
    return k == key and pid.isdigit() and start != "None" and _proc_start(int(pid)) == start


def _unlink(p: Path) -> None:
    try:
        p.unlink()
    except FileNotFoundError:
        pass


def join(rank: int, world: int, key: str | None = None, timeout_s: float | None = None) -> None:
    """All-ranks-present barrier ahead of RCCL: every rank publishes a join
    marker (job key, pid, process start time), then waits until all `world`
    markers of this job key name running processes. RCCL's bootstrap is entered
    only once every peer is known to be alive (a communicator whose peer never
    arrives blocks inside RCCL's bootstrap, and its abort can block too;
    DESIGN.md §6). A rank that does not arrive within the bound ends every
    other rank here with RendezvousError (ECOMM). A rank removes its own marker
    when it fails here and when its process exits, so a stale marker never
    stands in for a live peer of a later job with the same key."""
    key = key or job_key()
    timeout_s = default_timeout_s() if timeout_s is None else timeout_s
    mine = join_path(key, rank)
    tmp = mine.with_name(mine.name + f".{os.getpid()}.tmp")
    tmp.write_bytes(_marker(key))
    os.replace(tmp, mine)
    atexit.register(_unlink, mine)
    deadline = time.monotonic() + timeout_s
    missing = list(range(world))
    while True:
        missing = [r for r in missing if not marker_alive(join_path(key, r), key)]
        if not missing:
            return
        if time.monotonic() >= deadline:
            _unlink(mine)
            raise RendezvousError(f"rendezvous: rank {rank} of {world}: rank(s) {missing} never joined "
                                  f"within {timeout_s:g} s (job key {key}); no communicator was created")
        time.sleep(0.01)


def cleanup(key: str | None = None, world: int = 0) -> None:
    """Remove the job's unique-id file and its join markers (rank 0, once every
    rank has passed the communicator's first barrier)."""
    key = key or job_key()
    for p in [uid_path(key)] + [join_path(key, r) for r in range(world)]:
        _unlink(p)
