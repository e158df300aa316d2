"""ctypes binding of the native host runtime ``_runtime.so`` (csrc/runtime/*.cpp, built by ``make``).

The runtime replaces the reference's TensorFlow input stack (tf.data TFRecord reader + windowing,
src/inputs.py:231-268,528-568), its Cython/C text preparation (scripts/local_text2tfrecord.pyx:45-97,
scripts/train_tokenizer.pyx:98-169) and the TF Saver's file IO (src/run/run.py:161-175) with one C ABI.
Every entry point reports failures through ``rt_last_error``; :func:`fail` turns that into
:class:`RuntimeErrorNative`.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB = None
_LOCK = threading.Lock()

c_ll = ctypes.c_longlong
c_int = ctypes.c_int
c_u32 = ctypes.c_uint32
c_vp = ctypes.c_void_p
c_cp = ctypes.c_char_p
P_ll = ctypes.POINTER(c_ll)
P_u32 = ctypes.POINTER(c_u32)
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_f32 = ctypes.POINTER(ctypes.c_float)
P_u8 = ctypes.POINTER(ctypes.c_uint8)
PP_u8 = ctypes.POINTER(P_u8)


class RuntimeErrorNative(RuntimeError):
    """an error reported by the native runtime (message from ``rt_last_error``)"""


class LoaderConfig(ctypes.Structure):
    """mirror of ``rt::LoaderConfig`` (csrc/runtime/loader.cpp)"""
    _fields_ = [("window", c_ll), ("shift", c_ll), ("batch", c_ll), ("shuffle_buffer", c_ll),
                ("seed", ctypes.c_uint64), ("cycle", ctypes.c_int32), ("repeat", ctypes.c_int32),
                ("verify_crc", ctypes.c_int32), ("mode", ctypes.c_int32)]


class FeatureIn(ctypes.Structure):
    """mirror of ``rt::FeatureIn`` (csrc/runtime/rt.h)"""
    _fields_ = [("key", c_cp), ("kind", ctypes.c_int32), ("data", c_vp), ("n", c_ll), ("offsets", P_ll)]


_SIGS = {
    "rt_last_error": (c_cp, []),
    "rt_crc32c": (c_u32, [c_vp, c_ll, c_u32]),
    "rt_masked_crc32c": (c_u32, [c_vp, c_ll]),
    "rt_reader_open": (c_vp, [c_cp, c_int]),
    "rt_reader_count": (c_ll, [c_vp]),
    "rt_reader_record": (c_ll, [c_vp, c_ll, PP_u8]),
    "rt_reader_close": (None, [c_vp]),
    "rt_writer_open": (c_vp, [c_cp]),
    "rt_writer_write": (c_int, [c_vp, c_vp, c_ll]),
    "rt_writer_write_example": (c_int, [c_vp, ctypes.POINTER(FeatureIn), c_int]),
    "rt_writer_close": (c_int, [c_vp]),
    "rt_example_encode": (c_ll, [ctypes.POINTER(FeatureIn), c_int, c_vp, c_ll]),
    "rt_example_feature": (c_int, [c_vp, c_ll, c_cp, P_ll]),
    "rt_example_int64": (c_ll, [c_vp, c_ll, c_cp, P_ll, c_ll]),
    "rt_example_float": (c_ll, [c_vp, c_ll, c_cp, P_f32, c_ll]),
    "rt_example_bytes": (c_ll, [c_vp, c_ll, c_cp, c_ll, PP_u8]),
    "rt_utf8_decode": (c_ll, [c_vp, c_ll, P_i32, c_ll]),
    "rt_loader_create": (c_vp, [ctypes.POINTER(LoaderConfig), ctypes.POINTER(c_cp), P_ll, c_int]),
    "rt_loader_destroy": (None, [c_vp]),
    "rt_loader_next": (c_int, [c_vp, P_i32]),
    "rt_loader_start": (None, [c_vp, ctypes.POINTER(P_i32), c_int]),
    "rt_loader_acquire": (c_int, [c_vp, c_ll]),
    "rt_loader_release": (None, [c_vp, c_int]),
    "rt_loader_stop": (None, [c_vp]),
    "rt_loader_state": (c_ll, [c_vp, P_ll, c_ll]),
    "rt_loader_restore": (c_int, [c_vp, P_ll, c_ll]),
    "rt_jsonl_to_text": (c_ll, [c_cp, c_cp, c_cp, c_int, c_int, c_int, P_ll]),
    "rt_text_to_tfrecords": (c_ll, [c_cp, c_cp, c_cp, c_ll, c_ll]),
    "rt_blob_chunk": (c_ll, []),
    "rt_blob_pieces": (c_ll, [c_int, P_ll]),
    "rt_blob_write": (c_int, [c_cp, c_int, ctypes.POINTER(c_vp), P_ll, P_ll, P_u32, c_int]),
    "rt_blob_read": (c_int, [c_cp, c_int, ctypes.POINTER(c_vp), P_ll, P_ll, P_u32, c_int]),
}


def lib() -> ctypes.CDLL:
    """the loaded runtime; raises if ``_runtime.so`` was not built (``make``)"""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            # OBST_RUNTIME_SO: an alternative build of the runtime (the sanitizer builds of `make asan` / `make tsan`)
            path = os.environ.get("OBST_RUNTIME_SO") or os.path.join(_HERE, "_runtime.so")
            if not os.path.exists(path):
                raise RuntimeErrorNative(f"native runtime {path} is missing: run `make` in the repository root")
            L = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _LIB = L
    return _LIB


def enc(s) -> bytes:
    return s if isinstance(s, bytes) else os.fsencode(s)


def last_error() -> str:
    msg = lib().rt_last_error()
    return msg.decode(errors="replace") if msg else ""


def fail(what: str):
    raise RuntimeErrorNative(f"{what}: {last_error()}")
