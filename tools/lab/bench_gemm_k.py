#!/usr/bin/env python3
"""K-dependence of the NT GEMM (per-tile prologue/epilogue overhead vs steady-state K loop) next to torch.matmul
(hipBLASLt) on the same shapes. Random bf16 operands; interleaved repetitions."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

SHAPES = [(32768, N, K) for N in (2048, 4096) for K in (1024, 2048, 4096, 8192)]


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    res = {}
    bufs = {}
    for M, N, K in SHAPES:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        bufs[(M, N, K)] = (A, B, C)
    for rep in range(3):
        for M, N, K in SHAPES:
            A, B, C = bufs[(M, N, K)]
            ops = (raw.Operand(A, 0, K), raw.Operand(B, 0, K), raw.Operand(C, 0, N))
            t1 = timeit(lambda: raw.gemm(*ops, M, N, K))
            t2 = timeit(lambda: torch.matmul(A, B.t(), out=C))
            f = 2 * M * N * K / 1e12
            res.setdefault((M, N, K), []).append((f / t1, f / t2))
    for k, v in res.items():
        v.sort()
        o, t = v[len(v) // 2]
        print(f"M={k[0]} N={k[1]} K={k[2]}: ours {o:7.1f} TF/s   hipBLASLt {t:7.1f} TF/s")


if __name__ == "__main__":
    main()
