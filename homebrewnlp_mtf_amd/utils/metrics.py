"""Metrics: JSONL stream + TensorBoard event files + parameter report (ref src/run/utils_run.py:32-113 add_summary /
analyze_model, src/run/run.py:123-132 scalar keys).

TensorBoard files are written without TensorFlow or the tensorboard package: an event file is a TFRecord stream
of ``Event`` protos (wall_time = 1 double, step = 2 int64, file_version = 3 string, summary = 5 {value = 1
{tag = 1, simple_value = 2 float}}), framed by the native TFRecord writer.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
import typing

import torch


def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 0x80:
        out.append((v & 0x7f) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def encode_event(step: int, wall_time: float, scalars: typing.Optional[typing.Dict[str, float]] = None,
                 file_version: typing.Optional[str] = None) -> bytes:
    ev = _varint((1 << 3) | 1) + struct.pack("<d", wall_time) + _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        ev += _ld(3, file_version.encode())
    if scalars:
        summary = b"".join(_ld(1, _ld(1, k.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(v)))
                           for k, v in scalars.items())
        ev += _ld(5, summary)
    return ev


class TensorBoardWriter:
    def __init__(self, logdir: str):
        from ..data.tfrecord import TFRecordWriter
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self.w = TFRecordWriter(self.path)
        self.w.write(encode_event(0, time.time(), file_version="brain.Event:2"))

    def scalars(self, step: int, values: typing.Dict[str, float]):
        self.w.write(encode_event(step, time.time(), values))

    def close(self):
        self.w.close()


class MetricsWriter:
    """rank-0 JSONL (one object per logged step) + optional TensorBoard"""

    def __init__(self, path: typing.Optional[str], tensorboard_dir: typing.Optional[str] = None, enabled: bool = True):
        self.enabled = enabled
        self.f = open(path, "a") if (enabled and path) else None
        self.tb = TensorBoardWriter(tensorboard_dir) if (enabled and tensorboard_dir) else None

    def write(self, step: int, values: typing.Dict[str, typing.Any]):
        if not self.enabled:
            return
        clean = {k: (float(v.item()) if isinstance(v, torch.Tensor) else v) for k, v in values.items()}
        if self.f:
            self.f.write(json.dumps(dict(step=int(step), time=time.time(), **clean)) + "\n")
            self.f.flush()
        if self.tb:
            self.tb.scalars(step, {k: v for k, v in clean.items() if isinstance(v, (int, float))})

    def close(self):
        if self.f:
            self.f.close()
        if self.tb:
            self.tb.close()


def analyze_model(store, path: typing.Optional[str] = None) -> str:
    """parameter report grouped by scope (ref utils_run.py:65-113 `analyze_model` / model_size.info)"""
    groups: typing.Dict[str, int] = {}
    for n, s in store.specs.items():
        parts = n.split("/")
        key = "/".join(parts[:3]) if len(parts) > 3 else "/".join(parts[:-1])
        n_el = 1
        for d in s.full_shape:
            n_el *= d
        groups[key] = groups.get(key, 0) + n_el
    total = sum(groups.values())
    lines = [f"{'scope':<60} {'params':>14} {'share':>7}"]
    for k, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        lines.append(f"{k:<60} {v:>14,} {100 * v / max(total, 1):>6.2f}%")
    lines.append(f"{'total':<60} {total:>14,}")
    lines.append(f"variables: {len(store.specs)}")
    text = "\n".join(lines)
    if path:
        with open(path, "w") as f:
            f.write(text + "\n")
    return text


def grad_norms(store) -> typing.Dict[str, float]:
    """--debug_grad: per-variable gradient L2 norms (the reference wires histograms that never fire)"""
    out = {}
    for n in store.order:
        out[f"grad_norm/{n}"] = float(store.grad_view(n).float().norm().item())
    return out
