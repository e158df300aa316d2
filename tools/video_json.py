#!/usr/bin/env python3
"""Video work splitting (ref scripts/chunk_video_json.py, scripts/split_video_json.py).

Input JSON files hold {"id": [...], "duration": [...]} (a file, or a folder of them).

    # group videos into chunks of at least MIN_DURATION (shuffled, seeded) -> {prefix}work_chunks.json
    python tools/video_json.py chunk videos.json 3600 --prefix out/
    # balance chunks (or single videos) over N workers by total duration -> {prefix}work_split_{i}.json
    python tools/video_json.py split out/work_chunks.json 8 --prefix out/
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import typing


def load(path: str) -> typing.Tuple[list, list]:
    paths = [os.path.join(path, p) for p in sorted(os.listdir(path))] if os.path.isdir(path) else [path]
    ids, dur = [], []
    for p in paths:
        d = json.load(open(p))
        ids += d["id"]
        dur += d["duration"]
    return ids, dur


def _total(d) -> float:
    return float(sum(d)) if isinstance(d, (list, tuple)) else float(d)


def split_equal(ids: list, duration: list, num: int, min_duration: float = 256):
    """greedy longest-first assignment to the currently lightest bin (ref video2tfrecord.py:169-185)"""
    order = sorted(zip(duration, ids), key=lambda x: _total(x[0]), reverse=True)
    out_ids: typing.List[list] = [[] for _ in range(num)]
    out_dur: typing.List[list] = [[] for _ in range(num)]
    sums = [0.0] * num
    for d, i in order:
        if _total(d) > min_duration or min_duration <= 0:
            k = min(range(num), key=lambda j: sums[j])
            out_ids[k].append(i)
            out_dur[k].append(d)
            sums[k] += _total(d)
    return out_ids, out_dur


def chunk(ids: list, duration: list, min_duration: float, seed: int = 0):
    videos = list(zip(ids, duration))
    rng = random.Random(seed)
    rng.shuffle(videos)
    chunks_i, chunks_d, ci, cd, s = [], [], [], [], 0.0
    for i, d in videos:
        ci.append(i)
        cd.append(d)
        s += _total(d)
        if s >= min_duration:
            chunks_i.append(ci)
            chunks_d.append(cd)
            ci, cd, s = [], [], 0.0
    if ci:
        chunks_i.append(ci)
        chunks_d.append(cd)
    return chunks_i, chunks_d


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("chunk")
    c.add_argument("load_path")
    c.add_argument("min_duration", type=float)
    c.add_argument("--prefix", default="")
    c.add_argument("--seed", type=int, default=0)
    s = sub.add_parser("split")
    s.add_argument("load_path")
    s.add_argument("split", type=int)
    s.add_argument("--prefix", default="")
    a = ap.parse_args(argv)
    ids, dur = load(a.load_path)
    if a.cmd == "chunk":
        ci, cd = chunk(ids, dur, a.min_duration, a.seed)
        for k, (i, d) in enumerate(zip(ci, cd)):
            print(f"chunk: {k} videos: {len(i)} duration: {sum(_total(x) for x in d)}")
        json.dump({"id": ci, "duration": cd}, open(f"{a.prefix}work_chunks.json", "w"))
    else:
        if dur and not isinstance(dur[0], list):
            ids = [[i] for i in ids]
        si, sd = split_equal(ids, dur, a.split, -1)
        for k, (i, d) in enumerate(zip(si, sd)):
            print(f"split: {k} chunks: {len(i)} duration: {sum(_total(x) for x in d)}")
            json.dump({"id": i, "duration": d}, open(f"{a.prefix}work_split_{k}.json", "w"))
    return 0


if __name__ == "__main__":
    sys.exit(main())
