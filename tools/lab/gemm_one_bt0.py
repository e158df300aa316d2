#!/usr/bin/env python3
"""Forward-GEMM shapes of the GPT-Neo-1.3B step on the K-contiguous ([N][K]) weight layout, one at a time with
progress output (isolates a slow or stuck hipBLASLt algorithm)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def run(name, fn, flops):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    first = time.perf_counter() - t
    t = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"{name:40s} first {first * 1e3:8.1f} ms  steady {dt * 1e3:7.2f} ms  {flops / dt / 1e12:7.0f} TF/s", flush=True)


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("M", 131072))
    r = lambda n: (torch.rand(n, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    for (N, K, bt) in ((4096, 2048, 0), (4096, 2048, 1), (2048, 4096, 0), (2048, 4096, 1)):
        A, W, C = r(M * K), r(K * N), torch.empty(M * N, device=dev, dtype=torch.bfloat16)
        bop = raw.Operand(W, 0, K) if bt == 0 else raw.Operand(W, 1, N)
        run(f"M{M} N{N} K{K} b_t{bt}", lambda: raw.gemm(raw.Operand(A, 0, K), bop, raw.Operand(C, 0, N), M, N, K),
            2 * M * N * K)
        Rr = r(M * N)
        run(f"M{M} N{N} K{K} b_t{bt} +R", lambda: raw.gemm(raw.Operand(A, 0, K), bop, raw.Operand(C, 0, N), M, N, K,
                                                            R=Rr), 2 * M * N * K)
        del A, W, C, Rr
    # q/k/v: shared A, three weights, batched output
    K, N = 4096, 2048
    A, W, C = r(M * K), r(3 * K * N), torch.empty(3 * M * N, device=dev, dtype=torch.bfloat16)
    for bt in (0, 1):
        bop = raw.Operand(W, 0, K, K * N) if bt == 0 else raw.Operand(W, 1, N, K * N)
        run(f"qkv batch3 M{M} N{N} K{K} b_t{bt}", lambda: raw.gemm(raw.Operand(A, 0, K, 0), bop,
                                                                    raw.Operand(C, 0, N, M * N), M, N, K, batch=(3, 1)),
            3 * 2 * M * N * K)
    del A, W, C
    K, N = 2048, 50304
    A, W, C = r(M * K), r(K * N), torch.empty(M * N, device=dev, dtype=torch.bfloat16)
    for bt in (0, 1):
        bop = raw.Operand(W, 0, K) if bt == 0 else raw.Operand(W, 1, N)
        run(f"logits M{M} N{N} K{K} b_t{bt}", lambda: raw.gemm(raw.Operand(A, 0, K), bop, raw.Operand(C, 0, N),
                                                                M, N, K), 2 * M * N * K)


if __name__ == "__main__":
    main()
