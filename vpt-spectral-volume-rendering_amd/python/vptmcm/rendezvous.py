"""Torch-free bootstrap of the RCCL communicator for one-process-per-GPU runs.

Under `torch.distributed.run` every local rank is a child of the same elastic
agent, so (parent pid, MASTER_PORT, run id) names the job uniquely on the
node. Rank 0 publishes the 128-byte ncclUniqueId through an atomically
renamed file in the temp dir; the other ranks poll for it. Everything after
that (barriers, max-over-ranks timing) runs over RCCL itself, so the
benchmark never loads a second HIP runtime (torch's) into the process.
Single node only, which is all the benchmark uses.
"""
from __future__ import annotations

import os
import tempfile
import time
from pathlib import Path


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


def cleanup(key: str | None = None) -> None:
    try:
        uid_path(key or job_key()).unlink()
    except FileNotFoundError:
        pass
