#!/usr/bin/env python3
"""Norm kernels on the GPT-Neo-1.3B step shape (131072 rows x 2048 features, bf16, scale + shift, residual-gradient
input R on the backward): time per call and effective HBM bandwidth (bytes the kernel must move / time)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    rows, F = int(os.environ.get("ROWS", 131072)), int(os.environ.get("F", 2048))
    groups = int(os.environ.get("GROUPS", 1))
    dev = torch.device("cuda")
    x = torch.randn(rows * F, device=dev).bfloat16()
    dy = torch.randn(rows * F, device=dev).bfloat16()
    r = torch.randn(rows * F, device=dev).bfloat16()
    sc = torch.randn(groups * F, device=dev) * 0.1 + 1
    sh = torch.randn(groups * F, device=dev) * 0.1
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    st = torch.empty(2 * rows, device=dev)
    dsc, dsh = torch.zeros_like(sc), torch.zeros_like(sh)
    us = timed(lambda: raw.norm_fwd(x, sc, sh, y, st, rows, F, groups))
    nb = rows * F * 2 * 2
    print(f"norm_fwd rows {rows} F {F}: {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s", flush=True)
    us = timed(lambda: raw.norm_bwd(x, dy, sc, st, dx, dsc, dsh, rows, F, groups, R=r))
    nb = rows * F * 2 * 4
    print(f"norm_bwd (+R, param grads) rows {rows} F {F}: {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s", flush=True)
    us = timed(lambda: raw.norm_bwd(x, dy, sc, st, dx, None, None, rows, F, groups, R=r))
    print(f"norm_bwd (+R, no param grads) rows {rows} F {F}: {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s", flush=True)
    us = timed(lambda: raw.norm_bwd(x, dy, sc, st, dx, None, None, rows, F, groups))
    nb = rows * F * 2 * 3
    print(f"norm_bwd (no R, no param grads) rows {rows} F {F}: {us:7.1f} us  {nb / us / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
