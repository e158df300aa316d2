#!/usr/bin/env python3
"""Video -> TFRecord frames for jannet mode (ref scripts/video2tfrecord.py `frame_encoder`, `worker`).

No downloader here (no network, no youtube-dl / OpenCV in this image): a "video" is a folder of frame images
(sorted by name) or a .npy array [T, H, W, C] uint8. Frames are resized to frame_width x frame_height, JPEG
encoded (PIL) and written one Example per frame:

    frame       bytes   JPEG image
    concat      int64   1 on the first frame of every video after the first in the same file
    tokens      int64   language_token_per_frame ids (subtitle text of the frame, padded)      [with --text]
    skip_frame  int64   1 for text-only frames                                                  [with --text]
    mask        int64   index of the last real token of the frame                               [with --text]

`--text` is a JSON file {video name: [per-frame strings]}; tokens are bytes (vocab 256) or ids of a tokenizers
JSON (`--tokenizer`). Words longer than the per-frame budget are split the way the reference's
bpe_with_word_split / char_level_encoder do: never more than language_token_per_frame - 1 tokens per frame.

    python tools/video2tfrecord.py --out data/vid/ --name demo --width 320 --height 176 videos/*
"""
from __future__ import annotations

import argparse
import io
import json
import os
import sys
import typing

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from homebrewnlp_mtf_amd.data.tfrecord import TFRecordWriter  # noqa: E402


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


def text_tokens(text: str, per_frame: int, padding: int, tokenizer=None) -> typing.Tuple[typing.List[int], int]:
    ids = list(text.encode()) if tokenizer is None else tokenizer.encode(text).ids
    ids = ids[:per_frame - 1]
    mask = len(ids)
    return ids + [padding] * (per_frame - len(ids)), mask


def write_videos(paths: typing.Sequence[str], out_path: str, width: int, height: int,
                 texts: typing.Optional[dict] = None, per_frame: int = 0, padding: int = 0, tokenizer=None) -> int:
    n = 0
    with TFRecordWriter(out_path) as w:
        for vi, path in enumerate(paths):
            key = os.path.basename(path.rstrip("/"))
            frame_text = (texts or {}).get(key, [])
            for fi, frame in enumerate(load_frames(path)):
                feat = {"frame": encode_jpeg(frame, width, height), "concat": [int(vi > 0 and fi == 0)]}
                if texts is not None:
                    t = frame_text[fi] if fi < len(frame_text) else ""
                    toks, mask = text_tokens(t, per_frame, padding, tokenizer)
                    feat.update(tokens=toks, skip_frame=[0], mask=[mask])
                w.write_example(feat)
                n += 1
    return n


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", required=True)
    ap.add_argument("--name", default="video")
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=176)
    ap.add_argument("--videos-per-file", type=int, default=8)
    ap.add_argument("--text", default=None)
    ap.add_argument("--language-token-per-frame", type=int, default=0)
    ap.add_argument("--padding-token", type=int, default=0)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("videos", nargs="+")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    texts = json.load(open(a.text)) if a.text else None
    tok = None
    if a.tokenizer:
        from tokenizers import Tokenizer
        tok = Tokenizer.from_file(a.tokenizer)
    for k in range(0, len(a.videos), a.videos_per_file):
        group = a.videos[k:k + a.videos_per_file]
        tmp = os.path.join(a.out, f".{a.name}_{k}.tmp")
        n = write_videos(group, tmp, a.width, a.height, texts, a.language_token_per_frame, a.padding_token, tok)
        os.replace(tmp, os.path.join(a.out, f"{a.name}_{k // a.videos_per_file:_>6d}_{n}.tfrecord"))
        print(f"{len(group)} videos, {n} frames", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
