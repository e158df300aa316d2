"""TensorFlow TensorBundle checkpoints (the reference's ``tf.train.Saver`` format, src/run/run.py:161-175,
src/run/utils_run.py:18-29) written and read without TensorFlow -- the MTF-layout interoperability path of SURVEY
§5.4 / N6.

A bundle ``<prefix>`` is two files:

* ``<prefix>.data-00000-of-00001`` -- the raw little-endian tensor bytes, back to back;
* ``<prefix>.index`` -- a LevelDB-format table (SSTable) mapping
  ``""`` -> ``BundleHeaderProto{num_shards, endianness, version}`` and every tensor name (bytewise sorted) ->
  ``BundleEntryProto{dtype, shape, shard_id, offset, size, crc32c}`` (crc32c = masked CRC32C of the tensor bytes).

The SSTable is built here: data blocks of prefix-compressed entries with a restart point every 16 keys, an empty
meta-index block, an index block (one entry per data block: last key -> varint block handle), every block followed by
a compression byte (0 = none) and the masked CRC32C of block + that byte, and the 48-byte footer ending in LevelDB's
magic number. CRC32C is the native SSE4.2 implementation (csrc/runtime/crc32c.cpp).

``export_checkpoint`` turns a native ``obst-ckpt-v1`` checkpoint (any TP degree: shards are concatenated along their
TP dim) into a bundle with the reference's variable / slot names plus ``global_step``; ``load_into`` reads a bundle
back into a trainer (re-sliced to its TP rank). Parity note: no TensorFlow (and no TF-written checkpoint in the
reference tree) is available here, so byte-level agreement with TF's reader is "parity unpinned"; the tests check
the wire format against the LevelDB / protobuf encoding rules and round-trip every dtype.
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
import typing

import numpy as np

from ..data import native as N

MAGIC = 0xdb4775248b80fb57
BLOCK_SIZE = 4096
RESTART_INTERVAL = 16
# tensorflow/core/framework/types.proto
DT = {np.dtype(np.float32): 1, np.dtype(np.float64): 2, np.dtype(np.int32): 3, np.dtype(np.uint8): 4,
      np.dtype(np.int16): 5, np.dtype(np.int8): 6, np.dtype(np.int64): 9, np.dtype(np.bool_): 10,
      np.dtype(np.uint16): 17, np.dtype(np.float16): 19}
DT_BFLOAT16 = 14
NP_OF_DT = {v: k for k, v in DT.items()}


def masked_crc32c(buf: bytes) -> int:
    b = bytes(buf)
    return int(N.lib().rt_masked_crc32c(ctypes.c_char_p(b), len(b)))


# ---- protobuf wire encoding ------------------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int) -> typing.Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v) if v else b""


def _field_bytes(num: int, b: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(b)) + b


def header_proto() -> bytes:
    """BundleHeaderProto{num_shards: 1, endianness: LITTLE (0, default), version: VersionDef{producer: 1}}"""
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1))


def entry_proto(dtype: int, shape: typing.Sequence[int], offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d)) if d else b"") for d in shape)
    return (_field_varint(1, dtype) + _field_bytes(2, dims) + _field_varint(4, offset) + _field_varint(5, size) +
            _varint((6 << 3) | 5) + struct.pack("<I", crc))


def parse_proto(buf: bytes) -> typing.Dict[int, list]:
    """generic wire-format parser: field number -> list of values (varint ints, bytes, fixed32/64 ints)"""
    out: typing.Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v, pos = buf[pos:pos + n], pos + n
        elif wt == 5:
            v, pos = struct.unpack_from("<I", buf, pos)[0], pos + 4
        elif wt == 1:
            v, pos = struct.unpack_from("<Q", buf, pos)[0], pos + 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(num, []).append(v)
    return out


def decode_entry(buf: bytes) -> dict:
    f = parse_proto(buf)
    shape = []
    if 2 in f:
        for d in parse_proto(f[2][0]).get(2, []):
            shape.append(parse_proto(d).get(1, [0])[0])
    return {"dtype": f.get(1, [0])[0], "shape": shape, "shard_id": f.get(3, [0])[0], "offset": f.get(4, [0])[0],
            "size": f.get(5, [0])[0], "crc32c": f.get(6, [0])[0]}


# ---- LevelDB table ---------------------------------------------------------------------------------------------
class _BlockBuilder:
    def __init__(self, restart_interval: int):
        self.buf = bytearray()
        self.restarts = [0]
        self.count = 0
        self.last = b""
        self.interval = restart_interval

    def add(self, key: bytes, value: bytes):
        shared = 0
        if self.count < self.interval:
            m = min(len(key), len(self.last))
            while shared < m and key[shared] == self.last[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.count = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value)) + key[shared:] + value
        self.last = key
        self.count += 1

    def finish(self) -> bytes:
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))

    def size(self) -> int:
        return len(self.buf) + 4 * len(self.restarts) + 4


def _write_block(f, data: bytes) -> bytes:
    off = f.tell()
    f.write(data)
    f.write(b"\0" + struct.pack("<I", masked_crc32c(data + b"\0")))
    return _varint(off) + _varint(len(data))


def write_table(path: str, items: typing.List[typing.Tuple[bytes, bytes]]):
    items = sorted(items)
    with open(path, "wb") as f:
        index = _BlockBuilder(1)
        blk = _BlockBuilder(RESTART_INTERVAL)
        last = None
        for k, v in items:
            blk.add(k, v)
            last = k
            if blk.size() >= BLOCK_SIZE:
                index.add(last, _write_block(f, blk.finish()))
                blk = _BlockBuilder(RESTART_INTERVAL)
        if blk.count or not items:
            index.add(last if last is not None else b"", _write_block(f, blk.finish()))
        meta = _write_block(f, _BlockBuilder(RESTART_INTERVAL).finish())
        idx = _write_block(f, index.finish())
        footer = (meta + idx).ljust(40, b"\0") + struct.pack("<II", MAGIC & 0xFFFFFFFF, MAGIC >> 32)
        f.write(footer)


def _parse_block(data: bytes) -> typing.List[typing.Tuple[bytes, bytes]]:
    nrest = struct.unpack_from("<I", data, len(data) - 4)[0]
    end = len(data) - 4 - 4 * nrest
    out, pos, last = [], 0, b""
    while pos < end:
        shared, pos = _read_varint(data, pos)
        nonshared, pos = _read_varint(data, pos)
        vlen, pos = _read_varint(data, pos)
        key = last[:shared] + data[pos:pos + nonshared]
        pos += nonshared
        out.append((key, data[pos:pos + vlen]))
        pos += vlen
        last = key
    return out


def _read_block(raw: bytes, handle: bytes, verify: bool = True) -> bytes:
    off, p = _read_varint(handle, 0)
    size, _ = _read_varint(handle, p)
    data = raw[off:off + size]
    trailer = raw[off + size:off + size + 5]
    if trailer[0] != 0:
        raise ValueError("compressed SSTable blocks are not supported")
    if verify and struct.unpack("<I", trailer[1:])[0] != masked_crc32c(data + b"\0"):
        raise ValueError(f"SSTable block at {off}: CRC mismatch")
    return data


def read_table(path: str, verify: bool = True) -> typing.List[typing.Tuple[bytes, bytes]]:
    raw = open(path, "rb").read()
    if len(raw) < 48 or struct.unpack_from("<Q", raw, len(raw) - 8)[0] != MAGIC:
        raise ValueError(f"{path}: not a LevelDB table (bad magic)")
    footer = raw[len(raw) - 48:len(raw) - 8]
    _, p = _read_varint(footer, 0)
    _, p = _read_varint(footer, p)           # meta-index handle (unused)
    start = p
    _, p = _read_varint(footer, p)
    _, p = _read_varint(footer, p)
    idx_handle = footer[start:p]
    items = []
    for _, h in _parse_block(_read_block(raw, idx_handle, verify)):
        items.extend(_parse_block(_read_block(raw, h, verify)))
    return items


# ---- bundles ---------------------------------------------------------------------------------------------------
def _as_numpy(t) -> typing.Tuple[np.ndarray, int]:
    """-> (little-endian array of the stored bytes, TF dtype enum); torch bfloat16 is stored as DT_BFLOAT16"""
    try:
        import torch
        if isinstance(t, torch.Tensor):
            t = t.detach().cpu().contiguous()
            if t.dtype == torch.bfloat16:
                return t.view(torch.int16).numpy().view(np.uint16), DT_BFLOAT16
            t = t.numpy()
    except ImportError:  # pragma: no cover
        pass
    a = np.asarray(t)
    if not a.flags.c_contiguous:      # (np.ascontiguousarray would turn a 0-dim scalar into shape [1])
        a = a.copy(order="C")
    if a.dtype not in DT:
        raise TypeError(f"dtype {a.dtype} has no TensorBundle mapping")
    return a.astype(a.dtype.newbyteorder("<"), copy=False), DT[a.dtype]


def write(prefix: str, tensors: typing.Dict[str, typing.Any]):
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    entries = []
    off = 0
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        for name, t in tensors.items():
            a, dt = _as_numpy(t)
            b = a.tobytes()
            f.write(b)
            entries.append((name.encode(), entry_proto(dt, a.shape, off, len(b), masked_crc32c(b))))
            off += len(b)
    write_table(prefix + ".index", [(b"", header_proto())] + entries)


def read(prefix: str, verify: bool = True) -> typing.Dict[str, np.ndarray]:
    """-> name -> array (DT_BFLOAT16 comes back as float32)"""
    items = read_table(prefix + ".index", verify)
    header = parse_proto(dict(items)[b""])
    if header.get(1, [1])[0] != 1:
        raise ValueError("multi-shard bundles are not supported")
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    out = {}
    for k, v in items:
        if k == b"":
            continue
        e = decode_entry(v)
        b = data[e["offset"]:e["offset"] + e["size"]]
        if verify and masked_crc32c(b) != e["crc32c"]:
            raise ValueError(f"{k.decode()}: data CRC mismatch")
        if e["dtype"] == DT_BFLOAT16:
            u = np.frombuffer(b, dtype="<u2").astype(np.uint32) << 16
            a = u.view(np.float32)
        else:
            a = np.frombuffer(b, dtype=NP_OF_DT[e["dtype"]].newbyteorder("<"))
        out[k.decode()] = a.reshape(e["shape"]).copy()
    return out


# ---- checkpoint conversion -------------------------------------------------------------------------------------
def export_checkpoint(ckpt_dir: str, prefix: str, include_slots: bool = True) -> int:
    """native obst-ckpt-v1 directory -> TensorBundle with full (TP-unsharded) tensors; returns the tensor count"""
    import torch

    from .checkpoint import FORMAT, _ShardReader
    meta = json.load(open(os.path.join(ckpt_dir, "meta.json")))
    if meta.get("format") != FORMAT:
        raise ValueError(f"{ckpt_dir}: unknown checkpoint format {meta.get('format')}")
    readers = [_ShardReader(ckpt_dir, b) for b in meta["shards"]]
    index0 = readers[0].index
    names = [n for n, i in index0.items() if include_slots or i["kind"] == "variable"]
    parts = [r.read(names) for r in readers]
    out: typing.Dict[str, typing.Any] = {}
    for n in sorted(names):
        info = index0[n]
        if info["tp_dim"] is not None and len(parts) > 1:
            out[n] = torch.cat([p[n] for p in parts], info["tp_dim"])
        else:
            out[n] = parts[0][n]
    out["global_step"] = np.asarray(int(meta["step"]), dtype=np.int64)
    write(prefix, out)
    return len(out)


def load_into(trainer, prefix: str, strict: bool = True) -> int:
    """copy a bundle's variables (and, when present, optimizer slots) into a trainer; returns global_step"""
    import torch

    from .checkpoint import _named_tensors
    tensors = read(prefix)
    named = _named_tensors(trainer)
    mesh = trainer.mesh
    missing = [n for n, (_, info) in named.items() if info["kind"] == "variable" and n not in tensors]
    if missing and strict:
        raise KeyError(f"bundle lacks {len(missing)} variables, e.g. {missing[:3]}")
    with torch.no_grad():
        for n, (dst, info) in named.items():
            if n not in tensors:
                continue
            src = torch.from_numpy(np.ascontiguousarray(tensors[n])).float()
            if info["tp_dim"] is not None and mesh.tp > 1 and list(src.shape) != list(dst.shape):
                k = src.shape[info["tp_dim"]] // mesh.tp
                src = src.narrow(info["tp_dim"], mesh.tp_rank * k, k)
            if list(src.shape) != list(dst.shape):
                raise ValueError(f"{n}: bundle shape {list(src.shape)} vs model {list(dst.shape)}")
            dst.copy_(src.to(dst.device, dst.dtype))
    trainer.store.sync_compute()
    step = int(tensors.get("global_step", np.asarray(0)))
    trainer.global_step = step
    return step
