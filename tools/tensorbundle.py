#!/usr/bin/env python3
"""TensorBundle (tf.train.Saver checkpoint) interoperability without TensorFlow.

    tensorbundle.py export <native ckpt dir | model_path> <out prefix> [--no-slots]
    tensorbundle.py inspect <prefix>            # name, dtype, shape of every entry

``export`` writes ``<prefix>.index`` + ``<prefix>.data-00000-of-00001`` with the reference's variable and optimizer
slot names (TP shards concatenated) and ``global_step``; a trainer loads one back with
``homebrewnlp_mtf_amd.utils.tensorbundle.load_into``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from homebrewnlp_mtf_amd.utils import checkpoint as ckpt  # noqa: E402
from homebrewnlp_mtf_amd.utils import tensorbundle as TB  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("export")
    e.add_argument("src")
    e.add_argument("prefix")
    e.add_argument("--no-slots", action="store_true")
    i = sub.add_parser("inspect")
    i.add_argument("prefix")
    a = ap.parse_args()
    if a.cmd == "export":
        src = a.src
        if not os.path.exists(os.path.join(src, "meta.json")):
            src = ckpt.latest(src)
            if src is None:
                raise SystemExit(f"no checkpoint under {a.src}")
        n = TB.export_checkpoint(src, a.prefix, include_slots=not a.no_slots)
        print(f"wrote {n} tensors from {src} to {a.prefix}.index / .data-00000-of-00001")
    else:
        for k, v in sorted(TB.read(a.prefix).items()):
            print(f"{k:80s} {str(v.dtype):8s} {list(v.shape)}")


if __name__ == "__main__":
    main()
