"""Process-group bring-up: one process per GPU (``torch.distributed.run`` sets RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_*). Backend ``nccl`` is RCCL on ROCm (xGMI inside the node); ``gloo`` for CPU runs and tests.
Replaces the reference's TPU resolver / session / device assignment (src/main.py:107-147)."""
from __future__ import annotations

import datetime
import os
import typing

import torch
import torch.distributed as dist

from ..config import ModelParameter
from . import state as pstate


def env_rank() -> typing.Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(params: ModelParameter, device: str = "auto") -> typing.Tuple[pstate.Mesh, torch.device]:
    """initialise the process group (if world > 1), pick the device, build and install the DP x TP mesh"""
    rank, local_rank, world = env_rank()
    use_cuda = device == "cuda" or (device == "auto" and torch.cuda.is_available())
    if use_cuda:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        timeout = datetime.timedelta(seconds=int(params.dist_timeout_s or 1800))
        if use_cuda:
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group("gloo", timeout=timeout)
    dp, tp = params.resolve_mesh(world)
    mesh = pstate.Mesh(dp=dp, tp=tp, rank=rank).build_groups()
    pstate.set_mesh(mesh)
    return mesh, dev


def shutdown():
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
