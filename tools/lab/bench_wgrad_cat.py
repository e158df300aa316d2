#!/usr/bin/env python3
"""k/q/v weight gradients of one attention layer (dW_j[K][N] = baseᵀ · dkqv[:, jN:(j+1)N], T = 131072 tokens):
three GEMMs on the column slices of the interleaved gradient (as in F._DotAttention) against one GEMM over the whole
3N-wide gradient into a [K][3N] scratch followed by the scatter into the three [K][N] blocks."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 131072))


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
    for K, N in ((4096, 2048), (2048, 2048)):
        baseT = (torch.rand(K * T, device=dev) * 2 - 1).to(torch.bfloat16)
        dkqv = (torch.rand(T * 3 * N, device=dev) * 2 - 1).to(torch.bfloat16)
        g = torch.zeros(3 * K * N, device=dev)
        tmp = torch.zeros(K * 3 * N, device=dev)
        f = 2 * T * K * 3 * N / 1e12

        def three():
            for j in range(3):
                raw.gemm(raw.Operand(baseT, 0, T), raw.Operand(dkqv[j * N:], 1, 3 * N),
                         raw.Operand(g[j * K * N:], 0, N), K, N, T)

        def one():
            raw.gemm(raw.Operand(baseT, 0, T), raw.Operand(dkqv, 1, 3 * N), raw.Operand(tmp, 0, 3 * N), K, 3 * N, T)

        def scatter():
            g.view(3, K, N).copy_(tmp.view(K, 3, N).permute(1, 0, 2))

        t3 = timeit(three)
        t1 = timeit(one)
        ts = timeit(scatter)
        print(f"K {K} N {N}: three GEMMs {t3 * 1e3:.3f} ms ({f / t3:.0f} TF/s); one [K][3N] GEMM {t1 * 1e3:.3f} ms "
              f"({f / t1:.0f} TF/s) + scatter {ts * 1e3:.3f} ms", flush=True)
        one()
        scatter()
        ref = g.clone()
        three()
        torch.cuda.synchronize()
        print("  max |diff| one+scatter vs three:", float((ref - g).abs().max()), flush=True)
        del baseT, dkqv, g, tmp


if __name__ == "__main__":
    main()
