#!/usr/bin/env python3
"""BPE tokenizer training (ref scripts/train_tokenizer.pyx:172-230).

Same recipe as the reference: every digit, whitespace character and ASCII punctuation character is its own
pre-token, everything else is split into runs (``Split(regex, 'isolated')``); a BPE model with unknown token
``\\x01``, the 256 single-byte characters as special tokens and ``--vocab-size`` (65536) entries. Input is the text
produced by ``tools/text2tfrecord.py prep``. Training runs in the Rust ``tokenizers`` library, as in the reference.

    python tools/train_tokenizer.py --out tokenizer.json data/txt/*.txt
"""
from __future__ import annotations

import argparse
import string
import sys


def build_tokenizer(cache_capacity: int = 2 ** 20):
    from tokenizers import Regex, Tokenizer
    from tokenizers.models import BPE
    from tokenizers.pre_tokenizers import Split
    split_chars = string.digits + " \t\n\r\x0b\x0c" + "".join("\\" + c for c in string.punctuation)
    tok = Tokenizer(BPE(unk_token="\x01", cache_capacity=cache_capacity, dropout=None))
    tok.pre_tokenizer = Split(Regex(f"[{split_chars}]|[^{split_chars}]+"), "isolated")
    return tok


def train(files, out, vocab_size=65536):
    from tokenizers.trainers import BpeTrainer
    tok = build_tokenizer()
    trainer = BpeTrainer(special_tokens=[chr(i) for i in range(256)], vocab_size=vocab_size)
    tok.train(files, trainer)
    tok.save(out, pretty=True)
    return tok


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="tokenizer.json")
    ap.add_argument("--vocab-size", type=int, default=65536)
    ap.add_argument("files", nargs="+")
    a = ap.parse_args(argv)
    train(a.files, a.out, a.vocab_size)
    print(f"wrote {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
