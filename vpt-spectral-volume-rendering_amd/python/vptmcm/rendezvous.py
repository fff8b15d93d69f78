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
    parts = [str(os.getppid()), os.environ.get("MASTER_PORT", "0"),
             os.environ.get("TORCHELASTIC_RUN_ID", "none")]
    return "-".join(p.replace("/", "_") for p in parts)


def uid_path(key: str) -> Path:
    return Path(tempfile.gettempdir()) / f"vptmcm-uid-{key}.bin"


def exchange_unique_id(rank: int, make_uid, key: str | None = None,
                       timeout_s: float = 180.0) -> bytes:
    """Rank 0 calls make_uid() and publishes it; others wait for it."""
    path = uid_path(key or job_key())
    if rank == 0:
        uid = make_uid()
        assert len(uid) == 128
        tmp = path.with_name(path.name + f".{os.getpid()}.tmp")
        tmp.write_bytes(uid)
        os.replace(tmp, path)
        return uid
    deadline = time.monotonic() + timeout_s
    while time.monotonic() < deadline:
        try:
            data = path.read_bytes()
            if len(data) == 128:
                return data
        except FileNotFoundError:
            pass
        time.sleep(0.02)
    raise TimeoutError(f"rank {rank}: no unique id at {path} after {timeout_s}s")


def cleanup(key: str | None = None) -> None:
    try:
        uid_path(key or job_key()).unlink()
    except FileNotFoundError:
        pass
