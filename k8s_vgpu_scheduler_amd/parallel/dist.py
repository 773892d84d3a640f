"""One process per GPU: environment-driven ``torch.distributed`` setup.

Reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT as set by
``torch.distributed.run`` (MASTER_ADDR defaults to 127.0.0.1: container
hostnames may not resolve).  On a GPU box the backend is ``nccl`` (= RCCL on
ROCm, xGMI peer-to-peer inside a node); without GPUs it is ``gloo`` so the same
code paths run in CPU tests.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int
    world: int
    local_rank: int
    backend: str
    device: torch.device

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_distributed(backend: str | None = None, timeout_s: float = 600.0) -> DistEnv:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    # dmabuf-only IPC on this driver: keep the legacy IPC path off for RCCL.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    gpu = torch.cuda.is_available() and backend != "gloo"
    backend = backend or ("nccl" if gpu else "gloo")
    device = torch.device(f"cuda:{local}") if backend == "nccl" else torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        import datetime

        kw = {"device_id": device} if backend == "nccl" else {}
        # MIVGPU_DIST_INIT (e.g. file:///tmp/rdzv) overrides env:// rendezvous:
        # tests use a file store so parallel runs never race for a TCP port
        init = os.environ.get("MIVGPU_DIST_INIT")
        if init:
            kw["init_method"] = init
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistEnv(rank, world, local, backend, device)


def shutdown():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
