#!/usr/bin/env python3
"""Output-projection (logits) GEMMs of the GPT-Neo-1.3B step through the framework's dispatch: forward
x[T][d] . Wt[V][d] -> [T][V], data gradient dlogits[T][V] . W -> [T][d], weight gradient xT[d][T] . dlogits[T][V]
(fp32) -- at the shipped padded vocabulary (50304) and at the next multiple of 256 (50432), and the weight gradient
in the token-strided x layout (no x transpose)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 131072))
D = 2048


def timeit(fn, n=6):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    dev = torch.device("cuda")
    r = lambda n: (torch.rand(n, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    x, xT = r(T * D), r(T * D)
    for V in (50304,):
        wt, w = r(V * D), r(D * V)
        lg = r(T * V)
        dx = torch.empty(T * D, device=dev, dtype=torch.bfloat16)
        gw = torch.zeros(D * V, device=dev, dtype=torch.float32)
        f = 2.0 * T * V * D / 1e12
        cases = (
            ("fwd  x.Wt", lambda: raw.gemm(raw.Operand(x, 0, D), raw.Operand(wt, 0, D), raw.Operand(lg, 0, V), T, V, D)),
            ("dgrad dl.W", lambda: raw.gemm(raw.Operand(lg, 0, V), raw.Operand(w, 0, V), raw.Operand(dx, 0, D), T, D, V)),
            ("wgrad xT.dl (NT)", lambda: raw.gemm(raw.Operand(xT, 0, T), raw.Operand(lg, 1, V), raw.Operand(gw, 0, V),
                                                  D, V, T)),
            ("wgrad x.dl (TT)", lambda: raw.gemm(raw.Operand(x, 1, D), raw.Operand(lg, 1, V), raw.Operand(gw, 0, V),
                                                 D, V, T)),
            # transposed product dWt[V][D] = dlᵀ . x: the vocabulary on M
            ("wgradT dl.xT", lambda: raw.gemm(raw.Operand(lg, 1, V), raw.Operand(xT, 0, T), raw.Operand(gw, 0, D),
                                              V, D, T)),
            ("wgradT dl.x", lambda: raw.gemm(raw.Operand(lg, 1, V), raw.Operand(x, 1, D), raw.Operand(gw, 0, D),
                                             V, D, T)),
        )
        for name, fn in cases:
            t = timeit(fn)
            print(f"V {V} {name:18s}: {t * 1e3:7.2f} ms {f / t:7.1f} TF/s", flush=True)
        del wt, w, lg, dx, gw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
