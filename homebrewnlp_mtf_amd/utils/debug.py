"""Debug / race-detection helpers.

* ``roctx`` ranges: with ``OBST_ROCTX=1`` every block, the optimizer step and the DP sync are wrapped in
  roctxRangePush/Pop (libroctx64 via ctypes) so `rocprofv3 --marker-trace` maps kernels to layers.
* collective-sequence check: with ``OBST_COLLECTIVE_CHECK=1`` every explicit collective folds (kind, numel, dtype)
  into a running hash; ``verify()`` all-gathers the hashes and raises on the first rank whose sequence diverged --
  the RevNet + TP + DP deadlock hazard of SURVEY §7.5 item 2, caught as an error instead of a hang.
* collective byte counter (always on, host arithmetic only): ``comm_bytes()`` returns the payload bytes per
  collective kind issued since the last ``comm_reset()`` -- ``bench.py`` prints bytes per step at N > 1.
"""
from __future__ import annotations

import contextlib
import ctypes
import hashlib
import os

import torch
import torch.distributed as dist

_ROCTX = None
_ROCTX_ON = os.environ.get("OBST_ROCTX", "0") == "1"
CHECK = os.environ.get("OBST_COLLECTIVE_CHECK", "0") == "1"
_hash = hashlib.sha256()
_count = 0
_bytes: dict = {}
_calls: dict = {}


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        try:
            lib = ctypes.CDLL("libroctx64.so")
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _ROCTX = lib
        except OSError:
            _ROCTX = False
    return _ROCTX


@contextlib.contextmanager
def range_(name: str):
    lib = _roctx() if _ROCTX_ON else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def record(kind: str, t: torch.Tensor):
    """count one collective's payload bytes; fold it into the sequence hash with OBST_COLLECTIVE_CHECK=1"""
    global _count
    _bytes[kind] = _bytes.get(kind, 0) + t.numel() * t.element_size()
    _calls[kind] = _calls.get(kind, 0) + 1
    if not CHECK:
        return
    _hash.update(f"{kind}:{t.numel()}:{t.dtype}|".encode())
    _count += 1


def verify(group=None) -> int:
    """all ranks must have issued the same collective sequence since the last verify; returns the count"""
    global _hash, _count
    if not CHECK or not dist.is_initialized():
        return _count
    mine = int.from_bytes(_hash.digest()[:7], "little")
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([mine, _count], dtype=torch.int64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    vals = [tuple(o.tolist()) for o in out]
    if any(v != vals[0] for v in vals):
        raise RuntimeError(f"collective sequence diverged across ranks (hash, count): {vals}")
    n = _count
    _hash = hashlib.sha256()
    _count = 0
    return n


def comm_bytes() -> dict:
    """{kind: [calls, payload bytes]} of the collectives recorded since the last ``comm_reset()``"""
    return {k: [_calls[k], _bytes[k]] for k in sorted(_bytes)}


def comm_reset():
    _bytes.clear()
    _calls.clear()
