#!/usr/bin/env python3
"""The MFMA phase GEMM (OBST_GEMM_LT=0) per operand layout: a large plain product in every (a_t, b_t), and the
token-mixer shape (2048 x 256 x 2048 per (b, h), 256 batches) dense and lower-triangular."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def rnd(n, dev):
    return (torch.rand(n, device=dev) * 2 - 1).to(torch.bfloat16)


def main():
    raw.lt_set(False)
    dev = torch.device("cuda")
    M = N = K = 8192
    A, B, C = rnd(M * K, dev), rnd(N * K, dev), torch.empty(M * N, device=dev, dtype=torch.bfloat16)
    for at in (0, 1):
        for bt in (0, 1):
            ops = (raw.Operand(A, at, K if at == 0 else M), raw.Operand(B, bt, K if bt == 0 else N),
                   raw.Operand(C, 0, N))
            t = timeit(lambda: raw.gemm(*ops, M, N, K))
            print(f"{M}^3 a_t {at} b_t {bt}: {t * 1e3:.3f} ms {2 * M * N * K / t / 1e12:.0f} TF/s", flush=True)
    del A, B, C
    Bt, S, H, Fd = 32, 2048, 8, 256
    hf = H * Fd
    W = rnd(H * S * S, dev)
    x = rnd(Bt * S * hf, dev)
    y = torch.empty_like(x)
    for tri in (0, 1):
        for bt in (1,):
            t = timeit(lambda: raw.gemm(raw.Operand(W, 0, S, 0, S * S), raw.Operand(x, 1, hf, S * hf, Fd),
                                        raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(Bt, H), tri=tri))
            fl = 2 * S * Fd * S * Bt * H * (0.5 if tri else 1.0)
            print(f"token mixer {S}x{Fd}x{S} x {Bt * H} batches tri {tri}: {t * 1e3:.3f} ms "
                  f"{fl / t / 1e12:.0f} TF/s (useful)", flush=True)


if __name__ == "__main__":
    main()
