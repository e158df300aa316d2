#!/usr/bin/env python3
"""Elementwise kernels at GPT-Neo-1.3B step sizes (T = 131072 tokens): gelu forward / backward on [T][4096], residual
add on [T][2048]; effective HBM bandwidth (bytes read + written / time)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 131072))


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    big = T * 4096
    x = torch.randn(big, device=dev).to(torch.bfloat16)
    z = torch.randn(big, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    for name, fn, n, arrays in (
            ("gelu fwd [T][4096]", lambda: raw.elementwise("act", x, y, act="gelu"), big, 2),
            ("gelu bwd [T][4096]", lambda: raw.elementwise("act_bwd", x, y, z=z, act="gelu"), big, 3),
            ("add [T][2048]", lambda: raw.elementwise("add", x[:T * 2048], y[:T * 2048], z=z[:T * 2048]), T * 2048, 3)):
        t = timeit(fn)
        print(f"{name}: {t * 1e6:.1f} us  {arrays * 2 * n / t / 1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
