#!/usr/bin/env python3
"""How much of a memory-bound kernel hides under a concurrent GEMM on MI355X: a hipBLASLt product of the step's
shape (131072 x 4096 x 2048) on one stream and the gelu backward / norm backward / weight-gradient GEMM on another,
timed sequentially and concurrently. Decides whether weight gradients on a side stream could pay in the backward."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = 131072


def main():
    dev = torch.device("cuda")
    r = lambda n: (torch.rand(n, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    x, w, y = r(T * 2048), r(4096 * 2048), r(T * 4096)
    z, dz, o = r(T * 4096), r(T * 4096), r(T * 4096)
    xT, dy2 = r(T * 2048), r(T * 2048)
    gw = torch.zeros(2048 * 2048, device=dev, dtype=torch.float32)

    def gemm():   # forward-shaped product on the K-contiguous weight
        raw.gemm(raw.Operand(x, 0, 2048), raw.Operand(w, 0, 2048), raw.Operand(y, 0, 4096), T, 4096, 2048)

    def gelu_bwd():
        raw.elementwise("act_bwd", z, o, z=dz, act="gelu")

    def wgrad():
        raw.gemm(raw.Operand(xT, 0, T), raw.Operand(dy2, 1, 2048), raw.Operand(gw, 0, 2048), 2048, 2048, T, beta=1.0)

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn, n=10):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e6

    for name, other, reps in (("gelu bwd [T][4096]", gelu_bwd, 3), ("wgrad 2048x2048xT", wgrad, 1)):
        ta = timed(gemm)
        tb = timed(other)

        def seq():
            gemm()
            for _ in range(reps):
                other()

        def conc():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                gemm()
            with torch.cuda.stream(s2):
                for _ in range(reps):
                    other()
            cur.wait_stream(s1)
            cur.wait_stream(s2)
        tsq, tcc = timed(seq), timed(conc)
        print(f"GEMM {ta:.0f} us + {reps} x {name} {tb:.0f} us: sequential {tsq:.0f} us, concurrent {tcc:.0f} us "
              f"(hidden {tsq - tcc:.0f} us of {reps * tb:.0f})", flush=True)


if __name__ == "__main__":
    main()
