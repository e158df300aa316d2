#!/usr/bin/env python3
"""Weight-gradient GEMMs of the GPT-Neo-1.3B step (fp32 out, K = T = 131072 tokens, few output tiles) through the
framework's dispatch with the split-K path (csrc/kernels/blaslt.cpp, OBST_LT_SPLITK) on and off, interleaved in one
process so clock drift hits both arms alike. Layouts: as the step issues them (profiles/r2_gemm_census.md) and
both-token-strided (no transposes)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 131072))


def timeit(fn, n=8):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    # (label, M, N, a_t, lda, b_t, ldb, beta)
    cases = (("kqv NT xT,dy[6144]", 4096, 2048, 0, T, 1, 6144, 1.0),
             ("d->2d NT", 2048, 4096, 0, T, 1, 4096, 1.0),
             ("2d->d TN x,dyT", 4096, 2048, 1, 4096, 0, T, 1.0),
             ("d->2d TT", 2048, 4096, 1, 2048, 1, 4096, 1.0),
             ("2d->d TT", 4096, 2048, 1, 4096, 1, 2048, 1.0),
             ("kqv TT", 2048, 2048, 1, 2048, 1, 6144, 1.0),
             ("kqv NT beta0", 2048, 2048, 0, T, 1, 6144, 0.0))
    for label, M, N, a_t, lda, b_t, ldb, beta in cases:
        A = (torch.rand(M * T if a_t == 0 else T * lda, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(T * ldb if b_t == 1 else N * ldb, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.zeros(M * N, device=dev, dtype=torch.float32)
        f = 2 * T * M * N / 1e12

        def run():
            raw.gemm(raw.Operand(A, a_t, lda), raw.Operand(B, b_t, ldb), raw.Operand(C, 0, N), M, N, T, beta=beta)
        res = {0: [], 1: []}
        for _ in range(3):
            for on in (0, 1):
                raw.lt_splitk_set(bool(on))
                res[on].append(timeit(run))
        raw.lt_splitk_set(True)
        t0, t1 = min(res[0]), min(res[1])
        print(f"{label:22s} M {M} N {N}: plain {t0 * 1e6:7.1f} us {f / t0:6.1f} TF/s | split {t1 * 1e6:7.1f} us "
              f"{f / t1:6.1f} TF/s", flush=True)
        del A, B, C
        torch.cuda.empty_cache()
    for cols in (2048, 4096):
        X = torch.empty(T * cols, device=dev, dtype=torch.bfloat16)
        Y = torch.empty_like(X)
        tt = timeit(lambda: raw.transpose(X, Y, T, cols, cols, T))
        print(f"transpose [{T}][{cols}]: {tt * 1e6:.1f} us")


if __name__ == "__main__":
    main()
