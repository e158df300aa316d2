"""Process-wide parallel state: the ``Mesh(dp, tp)`` of the current job.

The reference derives a TPU mesh ``b:{tpu/heads}, h:{heads}`` and lets Mesh-TensorFlow insert every collective
(``src/dataclass.py:247-252``). Here the grid is explicit: ``world = dp x tp`` with TP groups of
contiguous ranks (on one 8-GPU node every rank pair has a direct xGMI link, contiguous groups keep a TP group
inside a node when the job grows past one). Collectives are explicit RCCL calls (backend ``nccl`` is RCCL on
ROCm) issued from the autograd ops at the sites the reference's layout implied (X01-X12).
"""
from __future__ import annotations

import typing

import torch
import torch.distributed as dist


class Mesh:
    def __init__(self, dp: int = 1, tp: int = 1, rank: int = 0):
        self.dp, self.tp, self.rank = dp, tp, rank
        self.world = dp * tp
        self.tp_rank = rank % tp
        self.dp_rank = rank // tp
        self.tp_group: typing.Optional[dist.ProcessGroup] = None
        self.dp_group: typing.Optional[dist.ProcessGroup] = None
        self.world_group = None

    def build_groups(self):
        if not dist.is_initialized() or self.world == 1:
            return self
        self.world_group = dist.group.WORLD
        for d in range(self.dp):
            ranks = list(range(d * self.tp, (d + 1) * self.tp))
            g = dist.new_group(ranks)
            if self.rank in ranks:
                self.tp_group = g
        for t in range(self.tp):
            ranks = list(range(t, self.world, self.tp))
            g = dist.new_group(ranks)
            if self.rank in ranks:
                self.dp_group = g
        return self

    def __repr__(self):
        return f"Mesh(dp={self.dp}, tp={self.tp}, rank={self.rank})"


_MESH = Mesh()


def set_mesh(mesh: Mesh):
    global _MESH
    _MESH = mesh


def mesh() -> Mesh:
    return _MESH


def tp_size() -> int:
    return _MESH.tp


def tp_all_reduce(t: torch.Tensor, op=None) -> torch.Tensor:
    """In-place sum (or `op`) over the TP group; identity when tp == 1."""
    if _MESH.tp > 1 and t.device.type != "meta":   # the registration pass runs on meta tensors
        from ..utils import debug
        debug.record("tp_all_reduce", t)
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=_MESH.tp_group)
    return t


class _Done:
    def wait(self):
        return True


_DONE = _Done()


def tp_all_reduce_async(t: torch.Tensor):
    """Start an in-place sum over the TP group on RCCL's own stream (it orders itself after the compute stream's
    work so far) and return the handle; its ``wait()`` makes the compute stream wait for the collective without
    blocking the host. Work issued in between -- a layer's weight-gradient GEMM after its data-gradient all-reduce
    started -- runs on the compute stream while the collective moves over xGMI."""
    if _MESH.tp > 1 and t.device.type != "meta":
        from ..utils import debug
        debug.record("tp_all_reduce", t)
        return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=_MESH.tp_group, async_op=True)
    return _DONE


def _gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def tp_gather_rows(x: torch.Tensor, T: int, inner: int) -> torch.Tensor:
    """x [T, inner] -- this rank's contiguous block of the columns of a token-major [T, tp * inner] tensor (its heads)
    -> the whole [T, tp * inner]: one all-gather into [tp][T][inner] and one transposing copy"""
    tp = _MESH.tp
    if x.device.type == "meta":   # the registration pass
        return torch.empty(T, tp * inner, dtype=x.dtype, device="meta")
    from ..utils import debug
    debug.record("tp_all_gather", x)
    src = x.contiguous().view(-1)
    if _gloo(_MESH.tp_group):   # CPU rehearsal: gloo has no all_gather_into_tensor for every dtype
        parts = [torch.empty_like(src) for _ in range(tp)]
        dist.all_gather(parts, src, group=_MESH.tp_group)
        buf = torch.stack(parts)
    else:
        buf = torch.empty(tp * src.numel(), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(buf, src, group=_MESH.tp_group)
    return buf.view(tp, T, inner).transpose(0, 1).contiguous().view(T, tp * inner)


def tp_reduce_scatter_rows(y: torch.Tensor, T: int, inner: int) -> torch.Tensor:
    """y [T, tp * inner] partial sums -> this rank's block [T, inner] of their sum over the TP group"""
    tp = _MESH.tp
    if y.device.type == "meta":
        return torch.empty(T, inner, dtype=y.dtype, device="meta")
    from ..utils import debug
    debug.record("tp_reduce_scatter", y)
    src = y.view(T, tp, inner).transpose(0, 1).contiguous()
    if _gloo(_MESH.tp_group):   # gloo: all-reduce, keep this rank's block
        dist.all_reduce(src, group=_MESH.tp_group)
        return src[_MESH.tp_rank].contiguous()
    out = torch.empty(T * inner, dtype=y.dtype, device=y.device)
    dist.reduce_scatter_tensor(out, src.view(-1), group=_MESH.tp_group)
    return out.view(T, inner)
