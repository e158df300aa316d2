#!/usr/bin/env python3
"""Text → TFRecord data preparation (ref scripts/text2tfrecord.py, scripts/local_text2tfrecord.pyx,
scripts/train_tokenizer.pyx:98-169). Local filesystem only (no GCS / downloads).

    # 1. Pile-style jsonl(.zst|.gz) → normalised text (documents separated by chr(4)), native C++
    python tools/text2tfrecord.py prep --out data/txt/ data/pile/*.jsonl.zst
    # 2a. bytes records (UTF-8 code points are decoded by the loader), native C++
    python tools/text2tfrecord.py bytes --name pile --out data/tfr/ data/txt/*.txt
    # 2b. BPE int64 records with a local tokenizers JSON (tools/train_tokenizer.py)
    python tools/text2tfrecord.py int64 --name pile --tokenizer tokenizer.json --out data/tfr/ data/txt/*.txt

File names follow the reference: ``{int64|bytes}_{name}_{index:_>6}_{processed}_{count}.tfrecord`` (the trailing
count is what ``split_files`` / ``simulate_data_pipeline`` read). One Example{text} per file, ``--chunk-bytes``
(16 MiB default, BUFFER_SIZE in local_text2tfrecord.pyx:48) of text each.
"""
from __future__ import annotations

import argparse
import ctypes
import multiprocessing
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from homebrewnlp_mtf_amd.data import native as N  # noqa: E402
from homebrewnlp_mtf_amd.data.tfrecord import TFRecordWriter  # noqa: E402


def _prep_one(job):
    src, dst, key, sep, fix = job
    stats = (ctypes.c_longlong * 2)()
    n = N.lib().rt_jsonl_to_text(N.enc(src), N.enc(dst), key.encode(), sep, int(fix), 0, stats)
    if n < 0:
        raise RuntimeError(f"{src}: {N.last_error()}")
    return src, int(n), int(stats[0]), int(stats[1])


def prep(files, out, key="text", separator=4, fix_whitespace=True, procs=4):
    os.makedirs(out, exist_ok=True)
    jobs = []
    for i, f in enumerate(files):
        jobs.append((f, os.path.join(out, f"{i}.txt"), key, separator, fix_whitespace))
    with multiprocessing.Pool(procs) as pool:
        for src, n, inb, outb in pool.imap_unordered(_prep_one, jobs):
            print(f"{src}: {n} documents, {inb / 2 ** 20:.1f} MiB in, {outb / 2 ** 20:.1f} MiB out", flush=True)


def to_bytes(files, out, name, chunk_bytes):
    os.makedirs(out, exist_ok=True)
    index = 0
    for f in files:
        n = N.lib().rt_text_to_tfrecords(N.enc(f), N.enc(os.path.join(out, "")), name.encode(), chunk_bytes, index)
        if n < 0:
            raise RuntimeError(f"{f}: {N.last_error()}")
        index += int(n)
        print(f"{f}: {n} records", flush=True)
    return index


def _read_chunks(path, chunk_bytes):
    """chunks of text cut at the last newline (or UTF-8 boundary) before chunk_bytes"""
    with open(path, "rb") as f:
        carry = b""
        while True:
            data = carry + f.read(chunk_bytes - len(carry))
            if not data:
                return
            if len(data) < chunk_bytes:
                yield data.decode(errors="replace")
                return
            cut = data.rfind(b"\n") + 1 or len(data)
            while cut > 0 and cut < len(data) and (data[cut] & 0xC0) == 0x80:
                cut -= 1
            carry = data[cut:]
            yield data[:cut].decode(errors="replace")


def to_int64(files, out, name, tokenizer_path, chunk_bytes):
    from tokenizers import Tokenizer
    tok = Tokenizer.from_file(tokenizer_path)
    os.makedirs(out, exist_ok=True)
    index, processed = 0, 0
    for f in files:
        for text in _read_chunks(f, chunk_bytes):
            ids = tok.encode(text).ids
            processed += len(text)
            path = os.path.join(out, f"int64_{name}_{index:_>6d}_{processed}_{len(ids)}.tfrecord")
            with TFRecordWriter(path) as w:
                w.write_example({"text": ids})
            index += 1
        print(f"{f}: {index} records so far", flush=True)
    return index


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("prep")
    p.add_argument("--out", required=True)
    p.add_argument("--key", default="text")
    p.add_argument("--separator", type=int, default=4)
    p.add_argument("--no-fix", action="store_true")
    p.add_argument("--procs", type=int, default=4)
    p.add_argument("files", nargs="+")
    for name in ("bytes", "int64"):
        q = sub.add_parser(name)
        q.add_argument("--out", required=True)
        q.add_argument("--name", default="text")
        q.add_argument("--chunk-bytes", type=int, default=2 ** 24)
        if name == "int64":
            q.add_argument("--tokenizer", required=True)
        q.add_argument("files", nargs="+")
    a = ap.parse_args(argv)
    if a.cmd == "prep":
        prep(a.files, a.out, a.key, a.separator, not a.no_fix, a.procs)
    elif a.cmd == "bytes":
        to_bytes(a.files, a.out, a.name, a.chunk_bytes)
    else:
        to_int64(a.files, a.out, a.name, a.tokenizer, a.chunk_bytes)
    return 0


if __name__ == "__main__":
    sys.exit(main())
