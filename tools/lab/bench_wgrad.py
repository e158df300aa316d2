#!/usr/bin/env python3
"""Weight-gradient GEMM (dW[in][out] = X[T][in]^T dY[T][out], T = 32768) through the framework's hipBLASLt path in
every operand layout (token-strided = as produced; token-contiguous = after a transpose) and output dtype."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 32768))


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    for I, O in ((2048, 4096), (4096, 2048)):
        X = (torch.rand(T * I, device=dev) * 2 - 1).to(torch.bfloat16)
        dY = (torch.rand(T * O, device=dev) * 2 - 1).to(torch.bfloat16)
        XT = X.view(T, I).t().contiguous().view(-1)
        dYT = dY.view(T, O).t().contiguous().view(-1)
        f = 2 * T * I * O / 1e12
        for name, a, b in (("TT (as produced)", raw.Operand(X, 1, I), raw.Operand(dY, 1, O)),
                           ("NT (x transposed)", raw.Operand(XT, 0, T), raw.Operand(dY, 1, O)),
                           ("TN (dy transposed)", raw.Operand(X, 1, I), raw.Operand(dYT, 0, T)),
                           ("NN-K (both transposed)", raw.Operand(XT, 0, T), raw.Operand(dYT, 0, T))):
            for dt, beta in ((torch.float32, 1.0), (torch.float32, 0.0), (torch.bfloat16, 0.0)):
                C = torch.zeros(I * O, device=dev, dtype=dt)
                t = timeit(lambda: raw.gemm(a, b, raw.Operand(C, 0, O), I, O, T, beta=beta))
                print(f"in {I} out {O} {name:24s} {str(dt)[6:]:9s} beta {beta:.0f}: {t * 1e6:7.1f} us "
                      f"{f / t:7.1f} TF/s", flush=True)
        tt = timeit(lambda: raw.transpose(X, XT, T, I, I, T))
        print(f"transpose [{T}][{I}]: {tt * 1e6:.1f} us")


if __name__ == "__main__":
    main()
