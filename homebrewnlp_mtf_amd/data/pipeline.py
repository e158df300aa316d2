"""Text input pipeline: file sharding, run-log replay, the native windowed loader and the device feeder.

Reference: src/inputs.py -- ``split_files`` (:15-30), ``simulate_data_pipeline`` (:33-128), ``_text_decoder`` +
``decode_intstring`` / ``decode_bytestring`` (:231-268) and ``gpt_neo_input`` (:528-568).

MI355X-side design: the reference builds a tf.data graph per host and infeeds to TPU cores. Here every rank owns a
native loader (csrc/runtime/loader.cpp): a C++ thread decodes TFRecords, cuts ``ctx + patch`` windows with shift
``ctx``, runs the tf.data interleave/shuffle state machines and writes whole batches into pinned host buffers.
:class:`TextFeeder` issues the H2D copy of batch k+1 on a side HIP stream while step k computes, and carries the
loader's exact cursor with every batch (``consumed_state``) so checkpoints resume bit-exactly without the
reference's (never written) run log.
"""
from __future__ import annotations

import ctypes
import glob
import os
import random
import re
import typing

import numpy as np
import torch

from ..config import ModelParameter
from . import native as N

_COUNT_RE = re.compile(r"_(\d+)(?:\.tfrecord)?$")


def _element_count(path: str) -> int:
    """elements (tokens / characters) of a prepared file: the trailing ``_<count>.tfrecord`` of its name
    (ref simulate_data_pipeline, src/inputs.py:34)"""
    m = _COUNT_RE.search(os.path.basename(str(path)))
    if not m:
        raise ValueError(f"{path}: file name carries no element count (expected ..._<count>.tfrecord)")
    return int(m.group(1))


def split_files(filenames: typing.Sequence[str], slice_index: int, slice_count: int, seed: int,
                runs_log: typing.Optional[typing.Sequence[dict]] = None) -> typing.Tuple[typing.List[str], typing.List[int]]:
    """sorted file list, shuffled with Python's ``random`` when ``seed != 0`` (bit-compatible with the reference's
    ordering), optionally minus what earlier runs consumed, then every ``slice_count``-th file for this slice.
    Returns (files, per-file element skips)."""
    if not filenames:
        raise ValueError("no input files")
    files = sorted(filenames)
    if seed != 0:
        random.seed(seed)
        random.shuffle(files)
    skips = [0] * len(files)
    if runs_log:
        depleted, skips = simulate_data_pipeline(runs_log, files)
        keep = [i for i, d in enumerate(depleted) if not d]
        files = [files[i] for i in keep]
        skips = [skips[i] for i in keep]
    return files[slice_index::slice_count], skips[slice_index::slice_count]


def simulate_data_pipeline(runs_log: typing.Sequence[dict], file_list: typing.Sequence[str]
                           ) -> typing.Tuple[typing.List[bool], typing.List[int]]:
    """Replays earlier runs over the file list to find which files are used up and how many elements of the rest
    were consumed. Each run: {steps, ctx, slice_count, interleave_size, batch_size, grad_accumulation,
    token_patch_size}. Same accounting as the reference: per slice, files are taken in interleave groups; a group
    that holds fewer windows than the run still needs is consumed whole, otherwise windows of ``ctx`` elements are
    taken round-robin over the group's non-empty files. A file counts as skipped only if its whole interleave group
    is depleted."""
    sizes = [_element_count(f) for f in file_list]
    n = len(sizes)
    depleted = [False] * n
    used = [0] * n
    for run in runs_log:
        live = [i for i in range(n) if not depleted[i]]
        remaining = {i: sizes[i] - used[i] for i in live}
        slices = int(run["slice_count"])
        ctx = int(run["ctx"])
        patch = int(run["token_patch_size"])
        group = int(run["interleave_size"])
        need_total = int(run["steps"]) * int(run["grad_accumulation"]) * (int(run["batch_size"]) // slices)
        for s in range(slices):
            mine = live[s::slices]
            need = need_total
            for g0 in range(0, len(mine), group):
                ids = mine[g0:g0 + group]
                # usable elements: whole windows of ctx plus the patch of the final target
                usable = [remaining[i] - ((remaining[i] - patch) % ctx) - patch for i in ids]
                if sum(usable) // ctx > need:
                    left = list(usable)
                    k = 0
                    while sum(left) > 0 and need > 0:
                        while left[k] <= 0:
                            k = (k + 1) % len(left)
                        left[k] -= ctx
                        need -= 1
                        k = (k + 1) % len(left)
                    for j, i in enumerate(ids):
                        if left[j] <= 0:
                            depleted[i] = True
                        used[i] += usable[j] - left[j]
                else:
                    need -= sum(usable) // ctx
                    for j, i in enumerate(ids):
                        depleted[i] = True
                        used[i] = usable[j]
        # only groups whose files are all depleted are dropped
        for s in range(slices):
            idx = list(range(n))[s::slices]
            flags = depleted[s::slices]
            for g0 in range(0, len(idx), group):
                full = sum(flags[g0:g0 + group]) == group
                for i in idx[g0:g0 + group]:
                    depleted[i] = full
    return depleted, used


# ---------------------------------------------------------------------------------------------------------------
class TextLoader:
    """Batches of ``[batch, window]`` int32 token windows from TFRecord files (native loader).

    ``prefetch=0``: synchronous, every ``next()`` returns a fresh tensor. ``prefetch=n``: a native thread fills n
    (pinned, if a GPU is present) host buffers ahead; ``next()`` returns ``(buffer_index, view)`` and the caller
    gives the buffer back with ``release(buffer_index)``. The thread starts on the first ``next()`` so ``restore``
    can position the cursor first."""

    def __init__(self, files: typing.Sequence[str], window: int, shift: int, batch: int, cycle: int = 1,
                 skips: typing.Optional[typing.Sequence[int]] = None, repeat: bool = False, shuffle_buffer: int = 0,
                 seed: int = 0, prefetch: int = 0, verify_crc: bool = False, mode: int = 0, pin: bool = False):
        if not files:
            raise ValueError("TextLoader needs at least one file")
        self.window, self.batch, self.prefetch = int(window), int(batch), int(prefetch)
        cfg = N.LoaderConfig(int(window), int(shift), int(batch), int(shuffle_buffer), int(seed) & (2 ** 64 - 1),
                             int(cycle), int(bool(repeat)), int(bool(verify_crc)), int(mode))
        names = (N.c_cp * len(files))(*[N.enc(f) for f in files])
        sk = np.zeros(len(files), dtype=np.int64)
        if skips is not None:
            sk[:] = np.asarray(list(skips), dtype=np.int64)
        self.h = N.lib().rt_loader_create(ctypes.byref(cfg), names, sk.ctypes.data_as(N.P_ll), len(files))
        if not self.h:
            N.fail("loader")
        self.pin = pin and torch.cuda.is_available()
        self._bufs: typing.List[torch.Tensor] = []
        self._started = False

    def _start(self):
        self._bufs = [torch.empty(self.batch, self.window, dtype=torch.int32, pin_memory=self.pin)
                      for _ in range(self.prefetch)]
        ptrs = (N.P_i32 * self.prefetch)(*[ctypes.cast(b.data_ptr(), N.P_i32) for b in self._bufs])
        N.lib().rt_loader_start(self.h, ptrs, self.prefetch)
        self._started = True

    def next(self) -> typing.Optional[typing.Tuple[int, torch.Tensor]]:
        """(buffer index or -1, [batch, window] int32) or None at the end of the data"""
        L = N.lib()
        if self.prefetch <= 0:
            t = torch.empty(self.batch, self.window, dtype=torch.int32)
            r = L.rt_loader_next(self.h, ctypes.cast(t.data_ptr(), N.P_i32))
            if r < 0:
                N.fail("loader")
            return (-1, t) if r == 1 else None
        if not self._started:
            self._start()
        idx = L.rt_loader_acquire(self.h, -1)
        if idx == -2:
            N.fail("loader")
        if idx < 0:
            return None
        return idx, self._bufs[idx]

    def release(self, idx: int):
        if idx >= 0 and self.h:
            N.lib().rt_loader_release(self.h, int(idx))

    def state(self) -> np.ndarray:
        """the exact cursor after the last batch handed out (int64 vector)"""
        L = N.lib()
        n = int(L.rt_loader_state(self.h, None, 0))
        out = np.empty(n, dtype=np.int64)
        L.rt_loader_state(self.h, out.ctypes.data_as(N.P_ll), n)
        return out

    def restore(self, state) -> None:
        if self._started:
            raise RuntimeError("restore() must come before the first next() of a prefetching loader")
        st = np.ascontiguousarray(np.asarray(state, dtype=np.int64))
        if N.lib().rt_loader_restore(self.h, st.ctypes.data_as(N.P_ll), st.size) != 0:
            N.fail("loader restore")

    def __iter__(self):
        while True:
            r = self.next()
            if r is None:
                return
            idx, t = r
            if idx >= 0:
                t = t.clone()
                self.release(idx)
            yield t

    def close(self):
        if self.h:
            L = N.lib()
            if self._started:
                L.rt_loader_stop(self.h)
            L.rt_loader_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TextFeeder:
    """Turns loader windows into ``{"token_x", "token_y"}`` batches on ``device`` (ref gpt_neo_input _memory_func,
    src/inputs.py:543-551). On a GPU the H2D copy of the next batch runs on a side stream one step ahead; host
    buffers go back to the loader once their copy has completed."""

    def __init__(self, loader: TextLoader, params: ModelParameter, batch: int, device):
        self.loader = loader
        self.params = params
        self.batch = batch
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self.consumed_state = loader.state()
        self._pending = None
        self._to_release: typing.List[typing.Tuple[int, typing.Any]] = []
        self._done = False

    def _fetch(self):
        r = self.loader.next()
        if r is None:
            return None
        idx, host = r
        st = self.loader.state()
        if self.cuda:
            with torch.cuda.stream(self.stream):
                dev = host.to(self.device, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            return dev, ev, idx, st
        dev = host.clone()
        self.loader.release(idx)
        return dev, None, -1, st

    def _split(self, x: torch.Tensor) -> typing.Dict[str, torch.Tensor]:
        p = self.params
        tp, off = p.token_patch_size, p.output_offset
        n = p.sequence_length // tp
        x = x.view(self.batch, n + off, tp).long()
        if off > 0:
            return {"token_x": x[:, :n].contiguous(), "token_y": x[:, off:n + off].contiguous()}
        return {"token_x": x.contiguous(), "token_y": x.contiguous()}

    def next(self) -> typing.Optional[typing.Dict[str, torch.Tensor]]:
        for idx, ev in self._to_release:
            ev.synchronize()
            self.loader.release(idx)
        self._to_release = []
        if self._done:
            return None
        if self._pending is None:
            self._pending = self._fetch()
        cur = self._pending
        if cur is None:
            self._done = True
            return None
        dev, ev, idx, st = cur
        if ev is not None:
            cs = torch.cuda.current_stream(self.device)
            cs.wait_event(ev)
            dev.record_stream(cs)
            if idx >= 0:
                self._to_release.append((idx, ev))
        self._pending = self._fetch()
        self.consumed_state = st
        return self._split(dev)

    def close(self):
        for idx, ev in self._to_release:
            ev.synchronize()
        self._to_release = []
        if self.cuda:
            self.stream.synchronize()
        self.loader.close()


class SyntheticText:
    """uniform random tokens of the configured shape (benchmarks / smoke runs without data)"""

    def __init__(self, params: ModelParameter, batch: int, device, seed: int = 0):
        self.params = params
        self.batch = batch
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.consumed_state = None

    def next(self) -> typing.Dict[str, torch.Tensor]:
        p = self.params
        tp = p.token_patch_size
        n = p.sequence_length // tp
        t = torch.randint(0, p.vocab_size, (self.batch, n + 1, tp), device=self.device, generator=self.gen)
        return {"token_x": t[:, :-1].contiguous(), "token_y": t[:, 1:].contiguous()}

    def close(self):
        pass


def dataset_files(params: ModelParameter, kind: typing.Optional[str] = None) -> typing.List[str]:
    """all files matched by ``dataset_configs`` paths (optionally only entries of one ``type``)"""
    out = []
    for ds in params.dataset_configs or []:
        d = ds if isinstance(ds, dict) else dict(ds)
        if kind is not None and d.get("type", "text") != kind:
            continue
        out.extend(sorted(glob.glob(d["path"])))
    return out


def text_input(params: ModelParameter, batch: int, dp_rank: int, dp_size: int, device, prefetch: int = 2,
               state=None, runs_log=None) -> TextFeeder:
    """the rank's text feeder (ref gpt_neo_input, src/inputs.py:528-568): files sharded over data-parallel ranks,
    windows of ``sequence_length + token_patch_size * output_offset`` tokens with shift ``sequence_length``,
    ``interleaved_datasets`` files interleaved, shuffle + repeat with ``use_random_dataloader``."""
    files = dataset_files(params)
    files, skips = split_files(files, dp_rank, dp_size, params.data_seed * int(bool(params.shuffle_input_filenames)),
                               runs_log)
    if not files:
        raise ValueError(f"data-parallel rank {dp_rank} of {dp_size} got no input files")
    rnd = bool(params.use_random_dataloader)
    dev = torch.device(device)
    loader = TextLoader(files, params.sequence_length + params.token_patch_size * params.output_offset,
                        params.sequence_length, batch, cycle=int(params.interleaved_datasets), skips=skips,
                        repeat=rnd, shuffle_buffer=int(params.shuffle_buffer) if rnd else 0,
                        seed=int(params.data_seed), prefetch=max(1, int(prefetch)), pin=dev.type == "cuda")
    if state is not None:
        loader.restore(state)
    return TextFeeder(loader, params, batch, dev)
