"""Autoregressive sampling and the interactive run modes (ref src/run/inference.py:15-133, src/interface.py;
SURVEY C08/C31, §3.4).

Sampling semantics follow the reference's language loop: for ``position`` in ``[initial_pos, end_iterations)``
the model reads the whole (causal) context, the logits get Gumbel noise scaled by the temperature
(``logits - T * log(-log(u))``, u from a counter-hash RNG, see ``_NoiseSeeds``), ``argmax`` over the vocabulary, and the prediction made at
``position - 1`` is written into ``token_x[position]`` (the shift-by-one of inference.py:94-96). Only the one needed
position goes through the output projection (``Model.logits(positions=...)``), which gives the same tokens as the
reference's full-sequence projection for causal bodies.

``CompletionEngine`` replaces the reference's Manager-dict ``InterfaceWrapper`` (interface.py:231-280): requests go
into an in-process queue and one GPU thread serves them in batches of up to ``max_batch`` prompts.
"""
from __future__ import annotations

import queue
import random
import threading
import typing

import numpy as np
import torch

from ..config import ModelParameter
from ..ops import raw as R
from ..utils.log import log


class ContextExhaustedError(ValueError):
    pass


class InvalidTokenError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------------------------
class Tokenizer:
    """Byte/char-level for vocabularies <= 256 (the reference's `chr`/`ord` path), otherwise a local HF
    ``tokenizers`` JSON file (``params.tokenizer_path``; the reference downloads GPT-2's, impossible offline)."""

    def __init__(self, params: ModelParameter):
        self.params = params
        self.bpe = None
        path = getattr(params, "tokenizer_path", None)
        if params.vocab_size > 256:
            if not path:
                raise ValueError("vocab_size > 256 needs `tokenizer_path` (a tokenizers JSON file)")
            from tokenizers import Tokenizer as HFTokenizer
            self.bpe = HFTokenizer.from_file(path)

    def encode(self, text: str) -> typing.List[int]:
        if self.bpe is None:
            return list(text.encode()) if self.params.vocab_size == 256 else [ord(c) for c in text]
        return self.bpe.encode(text).ids

    def decode(self, tokens: typing.Sequence[int]) -> str:
        if self.bpe is None:
            if self.params.vocab_size == 256:
                return bytes(int(t) & 0xff for t in tokens).decode(errors="replace")
            return "".join(chr(int(t)) for t in tokens)
        return self.bpe.decode([int(t) for t in tokens], skip_special_tokens=False)


def process_token_output(tokens: np.ndarray, padding_token: int = -1,
                         tokenizer: typing.Optional[Tokenizer] = None) -> typing.List[str]:
    """ref interface.py:61-88 (without argmax: callers pass token ids)"""
    tokens = np.asarray(tokens).reshape(tokens.shape[0], -1)
    out = []
    for row in tokens:
        row = row.tolist()
        if padding_token > -1 and padding_token in row:
            row = row[:row.index(padding_token)]
        if tokenizer is None or tokenizer.bpe is None:
            out.append("".join(chr(t) if t > 31 and t != 127 and t != 10 else " " for t in row))
        else:
            out.append(tokenizer.decode(row))
    return out


# ---------------------------------------------------------------------------------------------------------------
class _NoiseSeeds:
    """Per-call seeds of the sampling kernel's counter RNG (splitmix64 of a 64-bit counter: no generator state on
    the device, and the CPU oracle draws the same noise)"""

    def __init__(self, params: ModelParameter):
        self.base = int(params.seed) if getattr(params, "seed", None) is not None else 0
        self.calls = 0

    def next(self) -> int:
        self.calls += 1
        return (self.base * 0x9E3779B97F4A7C15 + self.calls * 0xD1B54A32D192ED03) & (2 ** 64 - 1)


class Sampler:
    def __init__(self, model, params: ModelParameter, device):
        self.model, self.params, self.device = model, params, torch.device(device)
        self.seeds = _NoiseSeeds(params)
        self.kv_cache = bool(getattr(params, "kv_cache", True))

    @torch.no_grad()
    def sample(self, token_x: torch.Tensor, initial_pos, temperature, end_iterations) -> torch.Tensor:
        """token_x [B, S, patch] int; per-row initial position / temperature / end (scalars or [B] tensors)."""
        x = token_x.to(self.device, torch.int32).contiguous().clone()
        B, S = x.shape[0], x.shape[1]

        def vec(v, dtype):
            t = torch.as_tensor(v, dtype=dtype, device=self.device)
            return t.expand(B).clone() if t.dim() == 0 else t.clone()
        pos = vec(initial_pos, torch.long).clamp(min=1)
        temp = vec(temperature, torch.float32)
        end = vec(end_iterations, torch.long).clamp(max=S)
        if self.kv_cache and self.model.supports_kv_cache():
            return self._sample_cached(x, pos, temp, end)
        while bool((pos < end).any()):
            active = pos < end
            src = (pos - 1).clamp(max=S - 1)
            logits = self.model.logits(x, positions=src)[:, 0]          # [B, patch, V] fp32
            P, V = logits.shape[1], logits.shape[2]
            pred = torch.empty(B * P, dtype=torch.int32, device=self.device)
            # Gumbel-argmax + write of the token at min(pos, S-1) for rows with pos < end: one kernel (K21)
            R.sample(logits.reshape(B * P, V).contiguous(), temp, pred, self.seeds.next(), x=x, pos=pos, end=end,
                     patch=P)
            pos = torch.where(active, pos + 1, pos)
        return x

    def _sample_cached(self, x, pos, temp, end):
        """Incremental decoding: one prefill forward over the context, then one single-token forward per step
        (KV caches, csrc/kernels/aux_ops.hip::decode_attn_kernel) -- the same tokens as the full recompute."""
        B, S = x.shape[0], x.shape[1]
        m = self.model
        try:
            logits = m.prefill(x, (pos - 1).clamp(max=S - 1))
        except NotImplementedError:
            self.kv_cache = False
            return self.sample(x, pos, temp, end)
        try:
            rows = torch.arange(B, device=self.device)
            # every active row advances one position per step, so the loop runs max(end - pos) steps: one host sync
            # here instead of an any(pos < end) read-back after every token
            steps = int((end - pos).clamp(min=0).max())
            for it in range(steps):
                active = pos < end
                P, V = logits.shape[2], logits.shape[3]
                pred = torch.empty(B * P, dtype=torch.int32, device=self.device)
                R.sample(logits.reshape(B * P, V).contiguous(), temp, pred, self.seeds.next(), x=x, pos=pos, end=end,
                         patch=P)
                pos = torch.where(active, pos + 1, pos)
                if it == steps - 1:
                    break
                cur = (pos - 1).clamp(max=S - 1)           # the token just written; inactive rows rewrite theirs
                logits = m.decode(x[rows, cur].unsqueeze(1), cur)
        finally:
            m.end_decode()
        return x


# ---------------------------------------------------------------------------------------------------------------
class VideoSampler:
    """Autoregressive jannet sampling with frame feedback (ref src/run/inference.py:22-64).

    For ``position`` in ``[initial_pos, end)`` the model reads the frames (and per-frame tokens) so far; the frame
    predicted at ``position`` (the model's estimate of frame ``position + 1``) is quantised back to the uint8 input
    encoding (re-folding bits when ``use_bit_fold_input_pipeline``) and written into slot ``position + 1``, and the
    Gumbel-argmax tokens of ``position`` into ``token_x[position + 1]``. The reference writes both into slot
    ``position`` (its own "todo: fix token shift for video"), which overwrites the prompt frame it just read; the
    rebuild shifts by one so prompt frames are never modified."""

    def __init__(self, model, params: ModelParameter, device):
        self.model, self.params, self.device = model, params, torch.device(device)
        self.seeds = _NoiseSeeds(params)

    def _to_input(self, frame_out: torch.Tensor) -> torch.Tensor:
        p = self.params
        q = (frame_out.float() * 255.0).round().clamp(0, 255)
        if p.use_bit_fold_input_pipeline:
            base = 2 ** p.bit_fold_value
            parts = q.clamp(max=base - 1).chunk(p.fold_count, -1)
            q = sum(part * base ** i for i, part in enumerate(parts))
        return q.to(torch.uint8)

    @torch.no_grad()
    def sample(self, batch: dict, initial_pos: int, temperature: float, end: typing.Optional[int] = None) -> dict:
        p = self.params
        frame = batch["frame"].to(self.device).clone()
        tok = batch.get("token_x")
        tok = tok.to(self.device).clone() if tok is not None else None
        T = frame.shape[1] - 1
        end = T if end is None else min(int(end), T)
        inputs = {k: v.to(self.device) for k, v in batch.items() if k not in ("frame", "token_x", "token_y")
                  and isinstance(v, torch.Tensor)}
        for pos in range(max(0, int(initial_pos)), end):
            frame_out, logits = self.model.predict(dict(inputs, frame=frame, token_x=tok))
            if pos + 1 <= T:
                frame[:, pos + 1] = self._to_input(frame_out[:, pos])
            if tok is not None and logits is not None and pos + 1 < tok.shape[1]:
                lg = logits[:, pos, ..., :p.vocab_size].float()
                rows = lg.numel() // lg.shape[-1]
                pred = torch.empty(rows, dtype=torch.int32, device=self.device)
                temp = torch.full((rows,), float(temperature), dtype=torch.float32, device=self.device)
                R.sample(lg.reshape(rows, lg.shape[-1]).contiguous(), temp, pred, self.seeds.next())
                tok[:, pos + 1] = pred.view(lg.shape[:-1]).to(tok.dtype)
        out = {"frame": frame}
        if tok is not None:
            out["token_x"] = tok
        return out


def render_video(samples: typing.Sequence[typing.Tuple[np.ndarray, typing.Optional[typing.List[str]]]],
                 count: int, params: ModelParameter, save_prefix: str = "", upscale: int = 4,
                 line_split: int = 2, text_color=(255, 0, 255), prompt_sample_color=(0, 128, 255)) -> str:
    """Side-by-side animated GIF of sampled videos (ref src/interface.py:13-58, which writes an MJPG .avi through
    OpenCV; OpenCV is not part of this stack, PIL is). ``samples`` is a list of (frames [T, H, W, C] in [0, 1],
    per-frame texts or None); frames are upscaled by nearest neighbour, per-frame text is drawn in
    ``language_token_per_frame // line_split`` character lines and, with autoregressive sampling, each frame is
    labelled "prompt" or "sample". Returns the written path."""
    from PIL import Image, ImageDraw
    images = []
    n_frames = len(samples[0][0])
    for idx in range(n_frames):
        cols = []
        for frames, texts in samples:
            f = np.asarray(frames[idx], dtype=np.float32)
            if f.ndim == 2:
                f = f[..., None]
            f = np.clip(f * (params.color_quantization_value - 1), 0, 255).astype(np.uint8)
            f = f.repeat(upscale, 0).repeat(upscale, 1)
            img = Image.fromarray(f[..., 0] if f.shape[-1] == 1 else f[..., :3])
            img = img.convert("RGB")
            draw = ImageDraw.Draw(img)
            if texts is not None and idx < len(texts):
                width = max(1, params.language_token_per_frame // line_split)
                for li, k in enumerate(range(0, len(texts[idx]), width)):
                    draw.text((10, img.height - 12 * (len(texts[idx]) // width + 1) + 12 * li),
                              texts[idx][k:k + width], fill=tuple(text_color))
            if params.use_autoregressive_sampling:
                label = "prompt" if idx < params.initial_autoregressive_position else "sample"
                draw.text((10, 10), label, fill=tuple(prompt_sample_color))
            cols.append(np.asarray(img))
        images.append(Image.fromarray(np.concatenate(cols, axis=1)))
    path = f"{save_prefix}_{count}.gif"
    images[0].save(path, save_all=True, append_images=images[1:], duration=1000, loop=0)
    return path


# ---------------------------------------------------------------------------------------------------------------
class CompletionEngine:
    """Thread-safe completion service over one model (``complete`` blocks; ``submit`` returns a future)."""

    def __init__(self, sampler: Sampler, params: ModelParameter, max_batch: int = 8):
        self.sampler, self.params, self.max_batch = sampler, params, max_batch
        self.q: "queue.Queue" = queue.Queue()
        self._stop = False
        self.thread = threading.Thread(target=self._loop, daemon=True)
        self.thread.start()

    def submit(self, query: typing.List[int], temperature: float, response_len: int):
        p = self.params
        iter_pos = len(query)
        if iter_pos >= p.sequence_length:
            raise ContextExhaustedError(f"context of {iter_pos} tokens exceeds {p.sequence_length}")
        if query and (max(query) >= p.vocab_size or min(query) < 0):
            raise InvalidTokenError(f"tokens must be in [0, {p.vocab_size})")
        fill = [random.randint(0, p.vocab_size - 1) for _ in range(p.sequence_length - iter_pos)]
        fut: "queue.Queue" = queue.Queue(maxsize=1)
        end = min(response_len + iter_pos, p.sequence_length)
        self.q.put((query + fill, iter_pos, float(temperature), end, fut))
        return fut

    def complete(self, query, temperature: float, response_len: int) -> np.ndarray:
        out = self.submit(query, temperature, response_len).get()
        if isinstance(out, BaseException):
            raise out
        return out

    def _loop(self):
        while not self._stop:
            try:
                first = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            items = [first]
            while len(items) < self.max_batch:
                try:
                    items.append(self.q.get_nowait())
                except queue.Empty:
                    break
            try:
                p = self.params
                toks = torch.tensor([it[0] for it in items], dtype=torch.int32).view(len(items), p.sequence_length, 1)
                out = self.sampler.sample(toks, [it[1] for it in items], [it[2] for it in items],
                                          [it[3] for it in items]).cpu().numpy()
                for it, row in zip(items, out):
                    it[4].put(row.reshape(-1)[it[1]:it[3]].astype(np.int64))
            except BaseException as e:  # noqa: BLE001 -- handed to the waiting caller
                for it in items:
                    it[4].put(e)

    def close(self):
        self._stop = True
        self.thread.join(timeout=5)


# ---------------------------------------------------------------------------------------------------------------
def run_query(engine: CompletionEngine, tokenizer: Tokenizer, params: ModelParameter, stream=None):
    """`query` run mode: prompts from stdin (ref interface.py:177-220)"""
    import sys
    stream = stream or sys.stdin
    while True:
        print("Enter Query:", flush=True)
        line = stream.readline()
        if not line:
            return
        q = tokenizer.encode(line.rstrip("\n"))
        if len(q) >= params.sequence_length:
            print(f"Query is too long: at most {params.sequence_length - 1} tokens, got {len(q)}.")
            continue
        out = engine.complete(q, params.sampling_temperature, params.sequence_length)
        print("Response:")
        print(process_token_output(out[None], tokenizer=tokenizer)[0].rstrip(), flush=True)


def run_debug(engine: CompletionEngine, params: ModelParameter) -> typing.List[float]:
    """`debug` run mode: the same random prompt N times at temperature 0 must give identical completions
    (ref interface.py:283-302)."""
    scores = []
    for idx in range(params.num_of_sample):
        query = [random.randint(0, params.vocab_size - 1) for _ in range(min(32, params.sequence_length - 8))]
        futs = [engine.submit(query, 0.0, params.sequence_length)
                for _ in range(int(params.equal_debugging_items_per_check))]
        base, *rest = [f.get() for f in futs]
        score = float(np.mean([np.mean(np.equal(base, o)) * 100 for o in rest])) if rest else 100.0
        print(f"test:{idx} similarity score: {score:6.2f}%")
        scores.append(score)
    return scores


def run_video_sample(sampler: VideoSampler, tokenizer: Tokenizer, params: ModelParameter,
                     batches: typing.Iterable[dict], save_prefix: str = "") -> typing.List[str]:
    """`sample` run mode for jannet (ref interface.py:101-150): sample after `initial_autoregressive_position` and
    render prompt + samples next to the ground truth."""
    pos = int(params.initial_autoregressive_position)
    paths = []
    for i, b in enumerate(batches):
        if i >= params.num_of_sample:
            break
        b1 = {k: v[:1] for k, v in b.items() if isinstance(v, torch.Tensor)}
        out = sampler.sample(b1, pos, params.sampling_temperature)
        model = sampler.model

        def frames(f):     # frame targets [T, ...] in the decoder's quantised scale, mapped to [0, 1]
            v = model._frames(f[0, 1:]).float() * 255.0
            return (v / max(1, params.color_quantization_value - 1)).cpu().numpy()

        def texts(t):
            if t is None:
                return None
            return [process_token_output(t[0, k].reshape(1, -1).cpu().numpy(), params.padding_token,
                                         tokenizer)[0] for k in range(t.shape[1])]
        cols = [(frames(b1["frame"]), texts(b1.get("token_x"))), (frames(out["frame"]), texts(out.get("token_x")))]
        cols = [(_unpatch(f, params), t) for f, t in cols]
        paths.append(render_video(cols, i, params, save_prefix=save_prefix))
        log(f"video sample {i} written to {paths[-1]}")
    return paths


def _unpatch(f: np.ndarray, params: ModelParameter) -> np.ndarray:
    """decoder frames [T, Hp(, Wp), C*p*p] -> images [T, H, W, C]: inverse of decode_frame's reshape/transpose
    (whose memory order is [p, p, Hp, Wp, C], ref src/inputs.py:181-198)"""
    T, p = f.shape[0], params.patch_size
    hp, wp, c = params.frame_height_patch, params.frame_width_patch, params.color_channels
    flat = f.reshape(T, -1)[:, :p * p * hp * wp * c]
    return flat.reshape(T, p, p, hp, wp, c).transpose(0, 3, 1, 4, 2, 5).reshape(T, hp * p, wp * p, c)


def run_sample(sampler: Sampler, tokenizer: Tokenizer, params: ModelParameter, batches: typing.Iterable[dict]):
    """`sample` / `debug_old` run modes: complete dataset prompts after `initial_autoregressive_position`
    (ref interface.py:101-174)."""
    pos = int(params.initial_autoregressive_position)
    for i, b in enumerate(batches):
        if i >= params.num_of_sample:
            return
        x = b["token_x"][:1]
        out = sampler.sample(x, pos, params.sampling_temperature, params.sequence_length).cpu().numpy()
        print(f"sample_idx: {i}")
        print("Prompt:")
        print(process_token_output(x[:, :pos - 1].cpu().numpy(), tokenizer=tokenizer)[0])
        print("Output:")
        print(process_token_output(out[:, pos:], tokenizer=tokenizer)[0].rstrip(), flush=True)
        log(f"sample {i} done")
