"""torchrun environment contract.

The reference is launched by ``torchrun`` (`entrypoint.sh:33-39`), which
exports RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / GROUP_RANK /
MASTER_ADDR / MASTER_PORT to each worker
(`$TORCH/distributed/elastic/agent/server/local_elastic_agent.py:306-321`).
The workers read them through the ``env://`` rendezvous
(`$TORCH/distributed/rendezvous.py:243-281`) and ``LOCAL_RANK`` directly
(`train.py:75`).  This module is the single parser of that contract.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    local_world_size: int = 1
    group_rank: int = 0
    master_addr: str = "127.0.0.1"
    master_port: int = 29500

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def launched(self) -> bool:
        """True when a launcher (torchrun or ours) exported the contract."""
        return "RANK" in os.environ and "WORLD_SIZE" in os.environ


def _int(env, key, default):
    v = env.get(key)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError as e:
        raise ValueError(f"environment variable {key}={v!r} is not an integer") from e


def read_env(env=None) -> DistEnv:
    env = os.environ if env is None else env
    world = _int(env, "WORLD_SIZE", 1)
    rank = _int(env, "RANK", 0)
    if not 0 <= rank < max(world, 1):
        raise ValueError(f"RANK={rank} outside [0, WORLD_SIZE={world})")
    return DistEnv(
        rank=rank,
        local_rank=_int(env, "LOCAL_RANK", 0),
        world_size=world,
        local_world_size=_int(env, "LOCAL_WORLD_SIZE", 1),
        group_rank=_int(env, "GROUP_RANK", 0),
        master_addr=env.get("MASTER_ADDR", "127.0.0.1"),
        master_port=_int(env, "MASTER_PORT", 29500),
    )


def ensure_single_process_env() -> None:
    """Allow ``python train.py`` without a launcher (world size 1).

    The reference requires torchrun; we default the contract so a bare run
    behaves like ``torchrun --nproc-per-node 1``.
    """
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("LOCAL_RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_WORLD_SIZE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # world 1: port 0 lets the TCPStore server bind an OS-assigned port (a probed "free" port can be
    # taken by another socket before the bind: EADDRINUSE, seen between back-to-back bench runs)
    os.environ.setdefault("MASTER_PORT", "0" if os.environ.get("WORLD_SIZE") == "1" else str(_free_port()))


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
