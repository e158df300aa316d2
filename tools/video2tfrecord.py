#!/usr/bin/env python3
"""Video (+ subtitles) -> TFRecord frames for jannet mode (behaviour of the reference's scripts/video2tfrecord.py:
`frame_encoder` :133-166, `split_equal` :169-185, `decode_vtt` :188-304, `bpe_with_word_split` :307-360,
`char_level_encoder` :363-371 and the frame loop of `worker` :632-723).

No downloader here (no network, no youtube-dl / OpenCV in this image): a "video" is a folder of frame images
(sorted by name) or a .npy array [T, H, W, C] uint8 recorded at --fps. Frames are resized to width x height, JPEG
encoded (PIL) and written one Example per frame:

    frame       bytes   JPEG image (a 1x1 white JPEG on text-only and separator frames)
    concat      int64   1 on the separator frame written between two videos of one file
    tokens      int64   language_token_per_frame ids                                             [with text]
    skip_frame  int64   1 for text-only frames (the tokens that did not fit the frame before)     [with text]
    mask        int64   number of real tokens in `tokens` (the rest is padding)                    [with text]

Text comes from a WebVTT file next to the video (<stem>.vtt; `--subtitles`), decoded to timed words
(`decode_vtt`): YouTube's word-timed captions (inline <hh:mm:ss.mmm><c> tags) keep each word's own stamp, plain cues
spread their duration evenly over their words. The words are tokenised as a whole text and the tokens re-split per
timed word (`bpe_with_word_split`, any tokenizers JSON via `--tokenizer`) or per character (`--encoder char`,
`char_level_encoder`). Every kept frame takes the tokens of the words stamped before the end of its time window;
beyond language_token_per_frame - 1 tokens the rest goes to extra text-only frames (skip_frame = 1), exactly as the
reference worker does. `--text` (JSON {video: [per-frame strings]}) is the simpler per-frame alternative.

Differences from the reference, on purpose: cue identifiers and blank lines are not read as caption text (the
reference's cue loop appends the next cue's number to the previous cue's text), `mm:ss.mmm` stamps are accepted,
and --target-fps 0 keeps every frame (the reference divides by zero there).

    python tools/video2tfrecord.py --out data/vid/ --name demo --width 320 --height 176 --subtitles \\
        --tokenizer tok.json --language-token-per-frame 4 videos/*
"""
from __future__ import annotations

import argparse
import io
import json
import os
import re
import sys
import typing

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from homebrewnlp_mtf_amd.data.tfrecord import TFRecordWriter  # noqa: E402

_STAMP = re.compile(r"(?:(\d+):)?(\d{1,2}):(\d{2})[.,](\d{3})")
_INLINE = re.compile(r"<((?:\d+:)?\d{1,2}:\d{2}[.,]\d{3})>")
_TAG = re.compile(r"</?c[^>]*>")


def _seconds(stamp: str) -> float:
    m = _STAMP.fullmatch(stamp.strip())
    if m is None:
        raise ValueError(f"bad WebVTT time stamp {stamp!r}")
    h, mi, s, ms = m.groups()
    return int(h or 0) * 3600 + int(mi) * 60 + int(s) + int(ms) / 1000.0


def decode_vtt(content: str) -> typing.Tuple[str, typing.List[str], typing.List[float]]:
    """WebVTT -> (text, timed word groups each with a leading space, stamp in seconds per group); text is the
    concatenation of the groups. Word-timed captions: a group is the text between two inline stamps, stamped with the
    stamp that closes it (the reference pairs each piece with the stamp at its end); text after the last stamp joins
    the last group. Plain cues: every word of a cue is its own group, stamped start + i * duration / n."""
    words: typing.List[str] = []
    stamps: typing.List[float] = []
    if _INLINE.search(content) and "<c>" in content:
        stream = " ".join(line for line in content.split("\n") if "<c>" in line)
        pieces = _INLINE.split(stream)      # text, stamp, text, stamp, ..., text
        for k in range(0, len(pieces) - 1, 2):
            w = " ".join(_TAG.sub(" ", pieces[k]).split())
            words.append(" " + w)
            stamps.append(_seconds(pieces[k + 1]))
        tail = " ".join(_TAG.sub(" ", pieces[-1]).split())
        if tail and words:
            words[-1] = words[-1] + " " + tail
        return "".join(words), words, stamps
    lines = content.split("\n")
    i = 0
    while i < len(lines):
        if " --> " not in lines[i]:
            i += 1
            continue
        a, b = lines[i].split(" --> ", 1)
        t0, t1 = _seconds(a), _seconds(b.split()[0])
        i += 1
        text = []
        while i < len(lines) and lines[i].strip() and " --> " not in lines[i]:
            text.append(lines[i].strip())
            i += 1
        cue = " ".join(" ".join(text).split()).split(" ") if text else []
        cue = [w for w in cue if w]
        for j, w in enumerate(cue):
            words.append(" " + w)
            stamps.append(t0 + j * (t1 - t0) / len(cue))
    return "".join(words), words, stamps


def split_equal(ids: typing.Sequence, durations: typing.Sequence[float], num: int, min_duration: float = 256
                ) -> typing.Tuple[typing.List[list], typing.List[list]]:
    """balance items over `num` workers by total duration: longest first, each to the least loaded worker; items of
    at most min_duration are dropped (unless min_duration <= 0)"""
    bins: typing.List[list] = [[] for _ in range(num)]
    dbins: typing.List[list] = [[] for _ in range(num)]
    load = [0.0] * num
    for d, i in sorted(zip(durations, ids), reverse=True):
        if min_duration > 0 and d <= min_duration:
            continue
        k = min(range(num), key=lambda j: (load[j], j))
        bins[k].append(i)
        dbins[k].append(d)
        load[k] += d
    return bins, dbins


class _Tokenizer:
    """encode(text) -> ids and decode(id) -> str over a tokenizers JSON, or raw bytes (vocab 256) without one"""

    def __init__(self, path: typing.Optional[str] = None):
        self.tok = None
        if path:
            from tokenizers import Tokenizer
            self.tok = Tokenizer.from_file(path)

    def encode(self, text: str) -> typing.List[int]:
        return list(text.encode()) if self.tok is None else self.tok.encode(text).ids

    def decode(self, i: int) -> str:
        return bytes([i]).decode("latin-1") if self.tok is None else self.tok.decode([i])


def bpe_with_word_split(enc, words: typing.Sequence[str], text: str) -> typing.List[typing.List[int]]:
    """tokenise the whole text once, then hand the tokens out to the timed word groups in order: a group takes
    tokens while each token's text (spaces removed) is the next piece of the group's text (spaces removed); a token
    spanning two groups goes to neither and ends the assignment there, as in the reference"""
    ids = enc.encode(text)
    pieces = [enc.decode(i).replace(" ", "") for i in ids]
    out: typing.List[typing.List[int]] = []
    k = 0
    for w in words:
        rest = w.replace(" ", "")
        group = []
        while k < len(ids) and pieces[k] in w and rest.startswith(pieces[k]):
            group.append(ids[k])
            rest = rest[len(pieces[k]):]
            k += 1
        out.append(group)
    return out


def char_level_encoder(words: typing.Sequence[str]) -> typing.List[typing.List[int]]:
    """one token (the code point) per character of each timed group, its leading space included"""
    return [[ord(c) for c in w] for w in words]


def load_frames(path: str) -> typing.Iterator[np.ndarray]:
    from PIL import Image
    if path.endswith(".npy"):
        for f in np.load(path, allow_pickle=False):
            yield f
        return
    for name in sorted(os.listdir(path)):
        if name.lower().endswith((".jpg", ".jpeg", ".png", ".bmp", ".gif")):
            yield np.asarray(Image.open(os.path.join(path, name)).convert("RGB"))


def encode_jpeg(frame: np.ndarray, width: int, height: int, quality: int = 90) -> bytes:
    from PIL import Image
    img = Image.fromarray(frame.astype(np.uint8))
    if img.size != (width, height):
        img = img.resize((width, height), Image.BILINEAR)
    buf = io.BytesIO()
    img.save(buf, format="JPEG", quality=quality)
    return buf.getvalue()


def padding_jpeg() -> bytes:
    return encode_jpeg(np.full((1, 1, 3), 255, np.uint8), 1, 1)


def text_tokens(text: str, per_frame: int, padding: int, tokenizer=None) -> typing.Tuple[typing.List[int], int]:
    """per-frame text mode: the frame's string, at most per_frame - 1 tokens (the last slot stays padding)"""
    ids = list(text.encode()) if tokenizer is None else tokenizer.encode(text).ids
    ids = ids[:per_frame - 1]
    mask = len(ids)
    return ids + [padding] * (per_frame - len(ids)), mask


def subtitle_examples(jpeg: bytes, window_end: float, groups: typing.List[typing.List[int]],
                      stamps: typing.List[float], per_frame: int, padding: int, pad_jpeg: bytes
                      ) -> typing.List[dict]:
    """the Examples of one kept frame: the tokens of every group stamped before window_end (consumed from the
    front of groups / stamps), per_frame - 1 per Example; the first carries the image, the rest are text-only"""
    buf: typing.List[int] = []
    while groups and stamps[0] < window_end:
        buf += groups.pop(0)
        stamps.pop(0)
    out = []
    step = per_frame - 1
    for s in range(0, len(buf), step):
        part = buf[s:s + step]
        out.append({"frame": pad_jpeg if s else jpeg, "concat": [0], "tokens": part + [padding] * (per_frame - len(part)),
                    "skip_frame": [int(s > 0)], "mask": [len(part)]})
    if not out:
        out.append({"frame": jpeg, "concat": [0], "tokens": [padding] * per_frame, "skip_frame": [0], "mask": [0]})
    return out


def write_videos(paths: typing.Sequence[str], out_path: str, width: int, height: int,
                 texts: typing.Optional[dict] = None, per_frame: int = 0, padding: int = 0, tokenizer=None,
                 subtitles: bool = False, encoder: str = "bpe", fps: float = 30.0, target_fps: float = 0.0,
                 concat_token: int = 0, skip_if_no_subtitles: bool = True) -> int:
    """write the videos of one file; returns the number of Examples"""
    n = 0
    pad = padding_jpeg()
    enc = tokenizer if isinstance(tokenizer, _Tokenizer) else _Tokenizer(None)
    with_text = texts is not None or subtitles
    wrote_video = False
    with TFRecordWriter(out_path) as w:
        for path in paths:
            key = os.path.basename(path.rstrip("/"))
            groups: typing.List[typing.List[int]] = []
            stamps: typing.List[float] = []
            if subtitles:
                vtt = os.path.splitext(path.rstrip("/"))[0] + ".vtt"
                if os.path.exists(vtt):
                    with open(vtt, encoding="utf-8") as f:
                        text, words, stamps = decode_vtt(f.read())
                    groups = char_level_encoder(words) if encoder == "char" else bpe_with_word_split(enc, words, text)
                elif skip_if_no_subtitles:
                    continue
            if wrote_video:   # separator between two videos of one file
                sep = {"frame": pad, "concat": [1]}
                if with_text:
                    sep.update(tokens=[concat_token] * per_frame, skip_frame=[0], mask=[per_frame])
                w.write_example(sep)
                n += 1
            split = (round(fps) / target_fps) if target_fps > 0 else 1.0
            frame_text = (texts or {}).get(key, [])
            kept = -1
            for fi, frame in enumerate(load_frames(path)):
                slot = int(fi // split)
                if slot == kept:
                    continue
                kept = slot
                jpeg = encode_jpeg(frame, width, height)
                if subtitles:
                    exs = subtitle_examples(jpeg, (fi + split) / fps, groups, stamps, per_frame, padding, pad)
                elif texts is not None:
                    toks, mask = text_tokens(frame_text[fi] if fi < len(frame_text) else "", per_frame, padding,
                                             None if enc.tok is None else enc.tok)
                    exs = [{"frame": jpeg, "concat": [0], "tokens": toks, "skip_frame": [0], "mask": [mask]}]
                else:
                    exs = [{"frame": jpeg, "concat": [0]}]
                for e in exs:
                    w.write_example(e)
                n += len(exs)
            wrote_video = True
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", required=True)
    ap.add_argument("--name", default="video")
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=176)
    ap.add_argument("--videos-per-file", type=int, default=8)
    ap.add_argument("--workers", type=int, default=1, help="output shards balanced by frame count (split_equal)")
    ap.add_argument("--fps", type=float, default=30.0, help="frame rate the input frames were recorded at")
    ap.add_argument("--target-fps", type=float, default=0.0, help="0: keep every frame")
    ap.add_argument("--text", default=None, help="JSON {video name: [per-frame strings]}")
    ap.add_argument("--subtitles", action="store_true", help="read <video stem>.vtt next to each video")
    ap.add_argument("--keep-without-subtitles", action="store_true")
    ap.add_argument("--encoder", choices=["bpe", "char"], default="bpe")
    ap.add_argument("--language-token-per-frame", type=int, default=0)
    ap.add_argument("--padding-token", type=int, default=0)
    ap.add_argument("--concat-token", type=int, default=0)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("videos", nargs="+")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    texts = json.load(open(a.text)) if a.text else None
    tok = _Tokenizer(a.tokenizer)
    videos = list(a.videos)
    if a.workers > 1:   # one shard list per worker, balanced by length (frames)
        lengths = [sum(1 for _ in load_frames(v)) for v in videos]
        shards, _ = split_equal(videos, lengths, a.workers, min_duration=0)
        videos = [v for s in shards for v in s]
    for k in range(0, len(videos), a.videos_per_file):
        group = videos[k:k + a.videos_per_file]
        tmp = os.path.join(a.out, f".{a.name}_{k}.tmp")
        n = write_videos(group, tmp, a.width, a.height, texts, a.language_token_per_frame, a.padding_token, tok,
                         subtitles=a.subtitles, encoder=a.encoder, fps=a.fps, target_fps=a.target_fps,
                         concat_token=a.concat_token, skip_if_no_subtitles=not a.keep_without_subtitles)
        if n == 0:
            os.remove(tmp)
            continue
        os.replace(tmp, os.path.join(a.out, f"{a.name}_{k // a.videos_per_file:_>6d}_{n}.tfrecord"))
        print(f"{len(group)} videos, {n} frames", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
