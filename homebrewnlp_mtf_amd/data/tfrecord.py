"""TFRecord files and ``tf.train.Example`` messages without TensorFlow or a protobuf library.

Framing (u64 length, masked CRC32C of the length, payload, masked CRC32C of the payload) and the Example wire
format are implemented natively (csrc/runtime/tfrecord.cpp); this module is the Python face used by the data
pipelines, the TensorBoard writer and the preparation tools. Reference users: ``tf.data.TFRecordDataset`` +
``tf.parse_single_example`` (src/inputs.py:147-157,208,251-268), ``tf.io.TFRecordWriter`` in
scripts/text2tfrecord.py / scripts/video2tfrecord.py.
"""
from __future__ import annotations

import ctypes
import typing

import numpy as np

from . import native as N

KIND_NONE, KIND_BYTES, KIND_FLOAT, KIND_INT64 = 0, 1, 2, 3


def crc32c(data: bytes, masked: bool = False) -> int:
    L = N.lib()
    if masked:
        return int(L.rt_masked_crc32c(data, len(data)))
    return int(L.rt_crc32c(data, len(data), 0))


def utf8_decode(data: bytes) -> np.ndarray:
    """UTF-8 -> code points (int32); invalid sequences become U+FFFD like ``tf.strings.unicode_decode``"""
    out = np.empty(len(data), dtype=np.int32)          # never more code points than bytes
    n = N.lib().rt_utf8_decode(data, len(data), out.ctypes.data_as(N.P_i32), len(out))
    return out[:n]


# ---- Example encoding -------------------------------------------------------------------------------------------
def _feature(key: str, value, keep: list) -> N.FeatureIn:
    f = N.FeatureIn()
    kb = key.encode()
    keep.append(kb)
    f.key = kb
    if isinstance(value, str):
        value = value.encode()
    if isinstance(value, (bytes, bytearray, memoryview)):
        value = [bytes(value)]
    if isinstance(value, (list, tuple)) and value and isinstance(value[0], (bytes, bytearray, str)):
        vals = [v.encode() if isinstance(v, str) else bytes(v) for v in value]
        blob = b"".join(vals)
        offs = np.zeros(len(vals) + 1, dtype=np.int64)
        np.cumsum([len(v) for v in vals], out=offs[1:])
        buf = ctypes.create_string_buffer(blob, max(1, len(blob)))
        keep.extend([buf, offs])
        f.kind, f.data, f.n, f.offsets = KIND_BYTES, ctypes.cast(buf, ctypes.c_void_p), len(vals), \
            offs.ctypes.data_as(N.P_ll)
        return f
    arr = np.asarray(value)
    if arr.dtype.kind == "f":
        arr = np.ascontiguousarray(arr, dtype=np.float32).reshape(-1)
        kind = KIND_FLOAT
    elif arr.dtype.kind in "iub" or arr.size == 0:
        arr = np.ascontiguousarray(arr, dtype=np.int64).reshape(-1)
        kind = KIND_INT64
    else:
        raise TypeError(f"feature {key!r}: unsupported value type {arr.dtype}")
    keep.append(arr)
    f.kind, f.data, f.n, f.offsets = kind, arr.ctypes.data, arr.size, None
    return f


def _features(feats: typing.Mapping[str, typing.Any]):
    keep: list = []
    arr = (N.FeatureIn * len(feats))(*[_feature(k, v, keep) for k, v in feats.items()])
    return arr, keep


def encode_example(feats: typing.Mapping[str, typing.Any]) -> bytes:
    """dict -> serialised ``tf.train.Example``. Values: bytes/str (one bytes value), list of bytes (BytesList),
    float arrays (FloatList) or integer sequences / arrays (Int64List)."""
    arr, keep = _features(feats)
    L = N.lib()
    n = int(L.rt_example_encode(arr, len(feats), None, 0))
    out = ctypes.create_string_buffer(max(1, n))
    L.rt_example_encode(arr, len(feats), out, n)
    del keep
    return out.raw[:n]


class Example:
    """read access to one serialised ``tf.train.Example`` (decoded natively, values copied out)"""

    def __init__(self, raw: bytes):
        self.raw = bytes(raw)

    def kind(self, key: str) -> typing.Tuple[int, int]:
        cnt = N.c_ll()
        k = N.lib().rt_example_feature(self.raw, len(self.raw), key.encode(), ctypes.byref(cnt))
        if k < 0:
            raise N.RuntimeErrorNative(f"malformed feature {key!r}")
        return int(k), int(cnt.value)

    def int64(self, key: str) -> np.ndarray:
        kind, n = self.kind(key)
        if kind != KIND_INT64:
            raise KeyError(f"{key!r} is not an int64 feature (kind {kind})")
        out = np.empty(n, dtype=np.int64)
        N.lib().rt_example_int64(self.raw, len(self.raw), key.encode(), out.ctypes.data_as(N.P_ll), n)
        return out

    def float(self, key: str) -> np.ndarray:
        kind, n = self.kind(key)
        if kind != KIND_FLOAT:
            raise KeyError(f"{key!r} is not a float feature (kind {kind})")
        out = np.empty(n, dtype=np.float32)
        N.lib().rt_example_float(self.raw, len(self.raw), key.encode(), out.ctypes.data_as(N.P_f32), n)
        return out

    def bytes_list(self, key: str) -> typing.List[bytes]:
        kind, n = self.kind(key)
        if kind != KIND_BYTES:
            raise KeyError(f"{key!r} is not a bytes feature (kind {kind})")
        L = N.lib()
        out = []
        ptr = N.P_u8()
        for i in range(n):
            ln = L.rt_example_bytes(self.raw, len(self.raw), key.encode(), i, ctypes.byref(ptr))
            out.append(ctypes.string_at(ptr, ln) if ln > 0 else b"")
        return out

    def get_int(self, key: str, default: int = 0) -> int:
        kind, n = self.kind(key)
        if kind == KIND_NONE or n == 0:
            return default
        return int(self.int64(key)[0])

    def text_tokens(self, key: str = "text") -> np.ndarray:
        """int64 token ids, or the code points of a UTF-8 bytes feature (ref decode_intstring / decode_bytestring,
        src/inputs.py:254-268)"""
        kind, _ = self.kind(key)
        if kind == KIND_INT64:
            return self.int64(key)
        if kind == KIND_BYTES:
            return utf8_decode(self.bytes_list(key)[0]).astype(np.int64)
        raise KeyError(f"no text feature {key!r}")


# ---- files -------------------------------------------------------------------------------------------------------
class TFRecordWriter:
    def __init__(self, path: str):
        self.path = path
        self.h = N.lib().rt_writer_open(N.enc(path))
        if not self.h:
            N.fail("TFRecord writer")

    def write(self, payload: bytes):
        if N.lib().rt_writer_write(self.h, payload, len(payload)) != 0:
            N.fail(f"TFRecord write {self.path}")

    def write_example(self, feats: typing.Mapping[str, typing.Any]):
        arr, keep = _features(feats)
        if N.lib().rt_writer_write_example(self.h, arr, len(feats)) != 0:
            N.fail(f"TFRecord write {self.path}")
        del keep

    def flush(self):
        pass  # records are written through on every call; close() flushes the stdio buffer

    def close(self):
        if self.h:
            r = N.lib().rt_writer_close(self.h)
            self.h = None
            if r != 0:
                N.fail(f"TFRecord close {self.path}")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RecordFile:
    """random access to the records of one TFRecord file (mmapped and indexed by the native reader on open; the
    length CRC of every record is always checked, the payload CRC when ``verify_crc``)"""

    def __init__(self, path: str, verify_crc: bool = True):
        self.path = path
        self.h = N.lib().rt_reader_open(N.enc(path), int(verify_crc))
        if not self.h:
            N.fail("TFRecord read")
        self.n = int(N.lib().rt_reader_count(self.h))

    def __len__(self):
        return self.n

    def __getitem__(self, i: int) -> bytes:
        ptr = N.P_u8()
        ln = N.lib().rt_reader_record(self.h, int(i), ctypes.byref(ptr))
        if ln < 0:
            raise IndexError(i)
        return ctypes.string_at(ptr, ln) if ln else b""

    def close(self):
        if self.h:
            N.lib().rt_reader_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


def read_records(path: str, verify_crc: bool = True) -> typing.Iterator[bytes]:
    f = RecordFile(path, verify_crc)
    try:
        for i in range(len(f)):
            yield f[i]
    finally:
        f.close()


def count_records(path: str) -> int:
    f = RecordFile(path, verify_crc=False)
    n = len(f)
    f.close()
    return n
