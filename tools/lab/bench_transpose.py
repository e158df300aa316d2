#!/usr/bin/env python3
"""Token-major activation transposes of the GPT-Neo-1.3B step ([131072][2048] and [131072][4096] bf16) and the
weight-copy shapes; effective HBM bandwidth (read + write)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


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
    for rows, cols in ((131072, 2048), (131072, 4096), (4096, 2048), (2048, 4096)):
        x = torch.randn(rows * cols, device=dev).to(torch.bfloat16)
        y = torch.empty_like(x)
        t = timeit(lambda: raw.transpose(x, y, rows, cols, cols, rows))
        assert torch.equal(y.view(cols, rows), x.view(rows, cols).t())
        print(f"transpose [{rows}][{cols}]: {t * 1e6:7.1f} us {4 * rows * cols / t / 1e12:.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
