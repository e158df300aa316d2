"""Video (jannet) input: frame decoding, the windowed/interleaved video source, the jannet text source and the
weighted mix of both.

Reference: src/inputs.py ``get_video_decoder`` (:131-228), ``dataset_text`` (:271-367), ``dataset_video``
(:370-483) and ``dataset`` (:486-525, ``sample_from_datasets``).

Frames are stored one ``tf.train.Example`` per frame (``frame`` JPEG/PNG bytes, ``concat``, ``skip_frame`` and, with
language, ``tokens`` / ``mask``; tools/video2tfrecord.py writes them). A sample is a window of
``sequence_length + time_patch`` consecutive frames of one file with shift ``sequence_length``; files are
interleaved ``interleaved_datasets`` at a time (tf.data interleave, block length 1). Decoding runs on a thread pool
(PIL releases the GIL) in a background producer; every batch carries the exact interleave cursor so a checkpoint
resumes on the next window.

Deliberate differences: the language mask uses the ``mask`` feature (the reference reads ``skip_frame`` there,
src/inputs.py:220, which makes only token 0 valid); ``skip_frame`` defaults to 0 when absent.
"""
from __future__ import annotations

import concurrent.futures
import glob
import io
import queue
import threading
import typing
import zlib

import numpy as np
import torch

from ..config import ModelParameter
from . import native as N
from . import tfrecord as T
from .pipeline import TextLoader, split_files

_MAGIC = 0x4f425354564944  # "OBSTVID"


def _frame_shape(p: ModelParameter, single: bool = False) -> typing.List[int]:
    """model frame shape (channels hold ``time_patch`` frames), or one decoded frame's with ``single``"""
    shape = [p.frame_height_patch, p.frame_width_patch] if p.three_axes else \
        [p.frame_height_patch * p.frame_width_patch]
    return shape + [p.channel_color_size // (p.time_patch if single else 1)]


def _frame_dtype(p: ModelParameter):
    return np.int64 if p.use_bit_fold_input_pipeline else np.uint8


def decode_frame(data: bytes, p: ModelParameter) -> np.ndarray:
    """encoded image -> patch layout (ref op_decod, src/inputs.py:181-198): [H, W, C] is viewed as
    [Hp, p, Wp, p, C], transposed to [p, p, Hp, Wp, C] and reshaped to [Hp*Wp (or Hp, Wp), p*p*C]; colours are
    quantised to ``color_quantization_value`` levels and, with the bit-fold pipeline, ``fold_count`` channel
    groups are packed into one integer per channel."""
    from PIL import Image
    img = np.asarray(Image.open(io.BytesIO(data)).convert("RGB" if p.color_channels == 3 else "L"))
    if img.ndim == 2:
        img = img[..., None]
    ps, hp, wp, c = p.patch_size, p.frame_height_patch, p.frame_width_patch, p.color_channels
    if img.shape[0] != hp * ps or img.shape[1] != wp * ps:
        raise ValueError(f"frame is {img.shape[1]}x{img.shape[0]}, expected {wp * ps}x{hp * ps}")
    q = int(p.color_quantization_value)
    if q != 256:
        img = np.round(img.astype(np.float32) * ((q - 1) / 255.0))
    img = img.astype(_frame_dtype(p))
    x = img.reshape(hp, ps, wp, ps, c).transpose(1, 3, 0, 2, 4)
    shape = _frame_shape(p, single=True)
    if p.use_bit_fold_input_pipeline:
        x = x.reshape(shape[:-1] + [p.fold_count, shape[-1]]).astype(np.int64)
        mult = (2 ** p.bit_fold_value) ** np.arange(p.fold_count, dtype=np.int64)
        return (x * mult[:, None]).sum(-2)
    return np.ascontiguousarray(x.reshape(shape))


class _Frame(typing.NamedTuple):
    frame: typing.Optional[bytes]
    concat: int
    skip: int
    tokens: typing.Optional[np.ndarray]
    mask: int


def _parse(raw: bytes, lpf: int) -> _Frame:
    ex = T.Example(raw)
    concat = ex.get_int("concat")
    skip = ex.get_int("skip_frame")
    tokens, mask = None, 0
    if lpf > 0:
        kind, n = ex.kind("tokens")
        tokens = np.zeros(lpf, dtype=np.int64)
        if kind == T.KIND_INT64 and n:
            v = ex.int64("tokens")[:lpf]
            tokens[:len(v)] = v
        mask = ex.get_int("mask")
    frame = None if (skip > 0 or concat > 0) else ex.bytes_list("frame")[0]
    return _Frame(frame, concat, skip, tokens, mask)


def _files_hash(files: typing.Sequence[str]) -> int:
    h = 0
    for f in files:
        h = zlib.crc32(f.encode(), h)
    return h


class _Interleave:
    """tf.data ``interleave(cycle_length, block_length=1)`` over per-file window sequences (same state machine as
    the native text loader); an element is (file index, first frame of the window)."""

    def __init__(self, counts: typing.Sequence[int], window: int, shift: int, cycle: int, repeat: bool):
        self.counts, self.window, self.shift = list(counts), window, shift
        self.cycle, self.repeat = max(1, cycle), repeat
        self.next_input = 0
        self.ci = 0
        self.slots: typing.List[typing.Optional[typing.List[int]]] = [None] * self.cycle   # [input, window idx]

    def _windows(self, file: int) -> int:
        n = self.counts[file]
        return 0 if n < self.window else (n - self.window) // self.shift + 1

    def _exhausted_input(self) -> bool:
        return not self.repeat and self.next_input >= len(self.counts)

    def next(self) -> typing.Optional[typing.Tuple[int, int]]:
        empty = 0
        while not self._exhausted_input() or any(s is not None for s in self.slots):
            s = self.slots[self.ci]
            if s is not None:
                f = s[0] % len(self.counts)
                if s[1] < self._windows(f):
                    out = (f, s[1] * self.shift)
                    s[1] += 1
                    self.ci = (self.ci + 1) % self.cycle
                    return out
                self.slots[self.ci] = None
                self.ci = (self.ci + 1) % self.cycle
                empty += 1
                if self.repeat and empty > 2 * len(self.counts) + self.cycle:
                    raise RuntimeError(f"no video file holds a full window of {self.window} frames")
            elif not self._exhausted_input():
                self.slots[self.ci] = [self.next_input, 0]
                self.next_input += 1
            else:
                self.ci = (self.ci + 1) % self.cycle
        return None

    def state(self) -> typing.List[int]:
        out = [self.next_input, self.ci]
        for s in self.slots:
            out += [0, 0, 0] if s is None else [1, s[0], s[1]]
        return out

    def restore(self, st: typing.Sequence[int]):
        self.next_input, self.ci = int(st[0]), int(st[1])
        for i in range(self.cycle):
            o, a, b = (int(v) for v in st[2 + 3 * i:5 + 3 * i])
            self.slots[i] = [a, b] if o else None


class VideoSource:
    """jannet video batches (ref dataset_video + _pre_func, src/inputs.py:370-483):
    frame [B, T+1, Hp*Wp (or Hp, Wp), C] uint8, token_x / token_y [B, T, lang_patch, token_patch] int64,
    txt_msk (bool, same shape), vid_msk_src / vid_msk_tgt / cat_mask_x / cat_mask_y [B, T] bool."""

    def __init__(self, files: typing.Sequence[str], params: ModelParameter, batch: int, device, workers: int = 4,
                 prefetch: int = 2, repeat: bool = True, cycle: typing.Optional[int] = None):
        if not files:
            raise ValueError("VideoSource needs at least one file")
        self.files = list(files)
        self.p = params
        self.batch = batch
        self.device = torch.device(device)
        self.window = params.sequence_length + params.time_patch
        self.lpf = int(params.language_token_per_frame) if params.use_language else 0
        self._readers: typing.Dict[int, T.RecordFile] = {}
        counts = [T.count_records(f) for f in self.files]
        self.inter = _Interleave(counts, self.window, params.sequence_length,
                                 int(cycle or params.interleaved_datasets), repeat)
        self.pool = concurrent.futures.ThreadPoolExecutor(max(1, workers))
        self.prefetch = max(1, prefetch)
        self._q: typing.Optional[queue.Queue] = None
        self._thread: typing.Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.consumed_state = self._state()

    # ---- cursor ----------------------------------------------------------------------------------------------------
    def _state(self) -> np.ndarray:
        head = [_MAGIC, len(self.files), _files_hash(self.files), self.inter.cycle, self.window]
        return np.asarray(head + self.inter.state(), dtype=np.int64)

    def restore(self, state) -> None:
        st = np.asarray(state, dtype=np.int64).tolist()
        if len(st) < 5 or st[0] != _MAGIC:
            raise N.RuntimeErrorNative("not a video source state")
        if st[1] != len(self.files) or st[2] != _files_hash(self.files) or st[3] != self.inter.cycle or \
                st[4] != self.window:
            raise N.RuntimeErrorNative("video source state belongs to a different file list / window / cycle")
        self._halt()
        self.inter.restore(st[5:])
        self.consumed_state = self._state()

    # ---- production ------------------------------------------------------------------------------------------------
    def _reader(self, f: int) -> T.RecordFile:
        r = self._readers.get(f)
        if r is None:
            if len(self._readers) > 4 * self.inter.cycle:
                for k in list(self._readers)[:len(self._readers) // 2]:
                    self._readers.pop(k).close()
            r = self._readers[f] = T.RecordFile(self.files[f], verify_crc=False)
        return r

    def _decode(self, fr: _Frame) -> np.ndarray:
        if fr.frame is None:
            return np.zeros(_frame_shape(self.p, single=True), dtype=_frame_dtype(self.p))
        return decode_frame(fr.frame, self.p)

    def _produce(self) -> typing.Optional[typing.Tuple[dict, np.ndarray]]:
        elems = []
        for _ in range(self.batch):
            e = self.inter.next()
            if e is None:
                return None
            elems.append(e)
        st = self._state()
        recs = [_parse(self._reader(f)[s + i], self.lpf) for f, s in elems for i in range(self.window)]
        frames = list(self.pool.map(self._decode, recs))
        return self._assemble(recs, frames), st

    def _assemble(self, recs: typing.List[_Frame], frames: typing.List[np.ndarray]) -> dict:
        p = self.p
        B, W, Tn = self.batch, self.window, p.time_patch_size
        fs = _frame_shape(p, single=True)
        tp = p.time_patch
        # [B, T+1, tp, spatial..., C] -> [B, T+1, spatial..., tp * C]: a time patch stacks its frames per patch
        frame = np.stack(frames).reshape([B, Tn + 1, tp] + fs)
        frame = np.moveaxis(frame, 2, -2).reshape([B, Tn + 1] + fs[:-1] + [tp * fs[-1]])
        first = np.arange(Tn + 1) * p.time_patch            # flags of the first frame of every time patch
        concat = np.asarray([r.concat for r in recs], dtype=np.int64).reshape(B, W)[:, first]
        skip = np.asarray([r.skip for r in recs], dtype=np.int64).reshape(B, W)[:, first]
        cat = concat == 0
        fm = skip == 0
        out = {"frame": frame, "vid_msk_src": fm[:, :Tn], "vid_msk_tgt": fm[:, 1:], "cat_mask_x": cat[:, :Tn],
               "cat_mask_y": cat[:, 1:]}
        if self.lpf:
            tok = np.stack([r.tokens for r in recs]).reshape(B, W, self.lpf)[:, first]
            rng = np.arange(self.lpf)
            msk = rng[None, None, :] <= np.asarray([r.mask for r in recs]).reshape(B, W)[:, first][..., None]
            shp = (B, Tn + 1, p.language_token_patch, p.token_patch_size)
            tok, msk = tok.reshape(shp), msk.reshape(shp)
            out.update(token_x=tok[:, :Tn], token_y=tok[:, 1:], txt_msk=msk[:, 1:])
        return out

    def _run(self):
        try:
            while not self._stop.is_set():
                item = self._produce()
                while not self._stop.is_set():
                    try:
                        self._q.put(item, timeout=0.1)
                        break
                    except queue.Full:
                        continue
                if item is None:
                    return
        except BaseException as e:  # noqa: BLE001 -- forwarded to the consumer
            self._q.put(e)

    def _halt(self):
        if self._thread is not None:
            self._stop.set()
            self._thread.join()
            self._thread = None
            self._stop.clear()
            # the producer ran ahead: rewind to what was consumed
            self.inter.restore(np.asarray(self.consumed_state).tolist()[5:])

    def next(self) -> typing.Optional[typing.Dict[str, torch.Tensor]]:
        if self._thread is None:
            self._q = queue.Queue(self.prefetch)
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()
        item = self._q.get()
        if isinstance(item, BaseException):
            raise item
        if item is None:
            self._q.put(None)
            return None
        batch, st = item
        self.consumed_state = st
        return _to_device(batch, self.device)

    def close(self):
        self._halt()
        self.pool.shutdown(wait=True)
        for r in self._readers.values():
            r.close()
        self._readers.clear()


def _to_device(batch: dict, device: torch.device) -> typing.Dict[str, torch.Tensor]:
    out = {}
    for k, v in batch.items():
        t = torch.from_numpy(np.ascontiguousarray(v))
        if device.type == "cuda":
            t = t.pin_memory().to(device, non_blocking=True)
        out[k] = t
    return out


class JannetTextSource:
    """text-only samples for jannet mode (ref dataset_text, src/inputs.py:271-367): windows of
    (T+1)*(lpf-1) tokens with shift T*(lpf-1) become one language row per frame with a padding token appended;
    frames are zero and masked out (vid_msk_* False, cat_mask_* True), txt_msk marks targets != concat_token."""

    def __init__(self, files: typing.Sequence[str], params: ModelParameter, batch: int, device, prefetch: int = 2):
        p = params
        if p.language_token_per_frame < 2:
            raise ValueError("jannet text needs language_token_per_frame >= 2")
        self.p, self.batch, self.device = p, batch, torch.device(device)
        row = p.language_token_per_frame - 1
        self.loader = TextLoader(files, (p.time_patch_size + 1) * row, p.time_patch_size * row, batch,
                                 cycle=int(p.interleaved_datasets), repeat=True,
                                 shuffle_buffer=int(p.shuffle_buffer), seed=int(p.data_seed),
                                 prefetch=max(1, prefetch))
        self.consumed_state = self.loader.state()

    def restore(self, state):
        self.loader.restore(state)
        self.consumed_state = self.loader.state()

    def next(self) -> typing.Optional[typing.Dict[str, torch.Tensor]]:
        r = self.loader.next()
        if r is None:
            return None
        idx, t = r
        x = t.numpy().astype(np.int64)
        self.loader.release(idx)
        self.consumed_state = self.loader.state()
        p, B, Tn = self.p, self.batch, self.p.time_patch_size
        x = x.reshape(B, Tn + 1, p.language_token_per_frame - 1)
        x = np.concatenate([x, np.full((B, Tn + 1, 1), p.padding_token, dtype=np.int64)], 2)
        x = x.reshape(B, Tn + 1, p.language_token_patch, p.token_patch_size)
        ty = x[:, 1:]
        out = {"frame": np.zeros([B, Tn + 1] + _frame_shape(p), dtype=_frame_dtype(p)),
               "token_x": x[:, :Tn], "token_y": ty, "txt_msk": ty != p.concat_token,
               "vid_msk_src": np.zeros((B, Tn), bool), "vid_msk_tgt": np.zeros((B, Tn), bool),
               "cat_mask_x": np.ones((B, Tn), bool), "cat_mask_y": np.ones((B, Tn), bool)}
        return _to_device(out, self.device)

    def close(self):
        self.loader.close()


class MixedSource:
    """``sample_from_datasets`` (ref src/inputs.py:515-517): every batch comes from one source drawn with the
    given weights by a counter-based generator, so the mix is reproducible and resumable."""

    def __init__(self, sources: typing.Sequence, weights: typing.Sequence[float], seed: int):
        self.sources = list(sources)
        w = np.asarray(weights, dtype=np.float64)
        self.cdf = np.cumsum(w / w.sum())
        self.seed = int(seed)
        self.k = 0

    @property
    def consumed_state(self) -> np.ndarray:
        parts = [np.asarray([len(self.sources), self.k], dtype=np.int64)]
        for s in self.sources:
            st = np.asarray(s.consumed_state, dtype=np.int64)
            parts += [np.asarray([st.size], dtype=np.int64), st]
        return np.concatenate(parts)

    def restore(self, state):
        st = np.asarray(state, dtype=np.int64)
        if int(st[0]) != len(self.sources):
            raise N.RuntimeErrorNative("mixed-source state has a different number of datasets")
        self.k = int(st[1])
        pos = 2
        for s in self.sources:
            n = int(st[pos])
            s.restore(st[pos + 1:pos + 1 + n])
            pos += 1 + n

    def next(self):
        u = np.random.default_rng([self.seed, self.k]).random()
        self.k += 1
        i = int(min(np.searchsorted(self.cdf, u, side="right"), len(self.sources) - 1))
        return self.sources[i].next()

    def close(self):
        for s in self.sources:
            s.close()


class SyntheticVideo:
    """random frames / tokens of the configured jannet shapes, all masks on"""

    def __init__(self, params: ModelParameter, batch: int, device, seed: int = 0):
        self.p, self.batch, self.device = params, batch, torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed))
        self.consumed_state = None

    def next(self) -> typing.Dict[str, torch.Tensor]:
        p, B, Tn, d = self.p, self.batch, self.p.time_patch_size, self.device
        hi = 2 ** (p.bit_fold_value * p.fold_count) if p.use_bit_fold_input_pipeline else 256
        fdt = torch.int64 if p.use_bit_fold_input_pipeline else torch.uint8
        frame = torch.randint(0, min(hi, 2 ** 31 - 1), [B, Tn + 1] + _frame_shape(p), device=d,
                              generator=self.gen).to(fdt)
        on = torch.ones(B, Tn, dtype=torch.bool, device=d)
        out = {"frame": frame, "vid_msk_src": on, "vid_msk_tgt": on, "cat_mask_x": on, "cat_mask_y": on}
        if p.use_language:
            tok = torch.randint(0, p.vocab_size, (B, Tn + 1, p.language_token_patch, p.token_patch_size), device=d,
                                generator=self.gen)
            out.update(token_x=tok[:, :Tn].contiguous(), token_y=tok[:, 1:].contiguous(),
                       txt_msk=torch.ones_like(tok[:, 1:], dtype=torch.bool))
        return out

    def close(self):
        pass


def jannet_input(params: ModelParameter, batch: int, dp_rank: int, dp_size: int, device, workers: int = 4):
    """the rank's jannet feeder (ref dataset, src/inputs.py:486-525): one source per ``dataset_configs`` entry
    (video, or text when ``use_language``), mixed by weight."""
    sources, weights = [], []
    seed = params.data_seed * int(bool(params.shuffle_input_filenames))
    for ds in params.dataset_configs or []:
        d = ds if isinstance(ds, dict) else dict(ds)
        kind = d.get("type", "text")
        if kind not in ("video", "text"):
            raise ValueError(f"{kind} is not a supported dataset type")
        files = sorted(glob.glob(d["path"]))
        if not files:
            raise ValueError(f"no files match {d['path']}")
        files, _ = split_files(files, dp_rank, dp_size, seed)
        if kind == "video":
            sources.append(VideoSource(files, params, batch, device, workers=workers))
        elif params.use_language:
            sources.append(JannetTextSource(files, params, batch, device))
        else:
            continue
        weights.append(float(d.get("weight", 1)))
    if not sources:
        raise ValueError("jannet mode needs at least one video (or, with use_language, text) dataset")
    if len(sources) == 1:
        return sources[0]
    return MixedSource(sources, weights, int(params.data_seed))
