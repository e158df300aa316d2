"""Python face of the native parallel blob IO (csrc/runtime/blobio.cpp): many buffers → one file, 4 KiB aligned,
64 MiB pieces written/read by a thread pool, one CRC32C per piece."""
from __future__ import annotations

import ctypes
import os
import typing

import numpy as np
import torch

from ..data import native as N

Buffer = typing.Union[np.ndarray, torch.Tensor]


def _ptr_size(b: Buffer) -> typing.Tuple[int, int]:
    if isinstance(b, torch.Tensor):
        if b.device.type != "cpu" or not b.is_contiguous():
            raise ValueError("blob IO needs contiguous CPU tensors")
        return b.data_ptr(), b.numel() * b.element_size()
    if not b.flags["C_CONTIGUOUS"]:
        raise ValueError("blob IO needs contiguous arrays")
    return b.ctypes.data, b.nbytes


def _threads() -> int:
    return max(1, min(16, (os.cpu_count() or 4)))


def write_blobs(path: str, bufs: typing.Sequence[Buffer], threads: typing.Optional[int] = None) -> dict:
    n = len(bufs)
    ps = [_ptr_size(b) for b in bufs]
    ptrs = (ctypes.c_void_p * n)(*[p for p, _ in ps])
    sizes = np.array([s for _, s in ps], dtype=np.int64)
    offsets = np.zeros(n, dtype=np.int64)
    L = N.lib()
    pieces = int(L.rt_blob_pieces(n, sizes.ctypes.data_as(N.P_ll)))
    crcs = np.zeros(max(1, pieces), dtype=np.uint32)
    r = L.rt_blob_write(N.enc(path), n, ptrs, sizes.ctypes.data_as(N.P_ll), offsets.ctypes.data_as(N.P_ll),
                        crcs.ctypes.data_as(N.P_u32), threads or _threads())
    if r != 0:
        N.fail("checkpoint write")
    return {"offsets": offsets.tolist(), "sizes": sizes.tolist(), "crcs": crcs[:pieces].tolist()}


def read_blobs(path: str, bufs: typing.Sequence[Buffer], meta: dict, verify: bool = True,
               threads: typing.Optional[int] = None):
    """``meta``: {"offsets": [...], "sizes": [...], "crcs": [...]} for exactly these blobs, in order (the CRC list is
    the concatenation of every blob's piece CRCs, see ``piece_crcs``)."""
    n = len(bufs)
    ps = [_ptr_size(b) for b in bufs]
    sizes = np.array(meta["sizes"], dtype=np.int64)
    if [s for _, s in ps] != sizes.tolist():
        raise ValueError("destination sizes do not match the checkpoint index")
    ptrs = (ctypes.c_void_p * n)(*[p for p, _ in ps])
    offsets = np.array(meta["offsets"], dtype=np.int64)
    crcs = np.array(meta["crcs"], dtype=np.uint32) if verify else None
    r = N.lib().rt_blob_read(N.enc(path), n, ptrs, sizes.ctypes.data_as(N.P_ll), offsets.ctypes.data_as(N.P_ll),
                             crcs.ctypes.data_as(N.P_u32) if crcs is not None else None, threads or _threads())
    if r != 0:
        N.fail("checkpoint read")


def piece_crcs(meta: dict) -> typing.List[typing.List[int]]:
    """splits the flat CRC list of ``write_blobs`` into one list per blob"""
    chunk = int(N.lib().rt_blob_chunk())
    out, k = [], 0
    for s in meta["sizes"]:
        c = max(1, -(-int(s) // chunk))
        out.append(meta["crcs"][k:k + c])
        k += c
    return out
