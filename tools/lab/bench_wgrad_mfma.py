#!/usr/bin/env python3
"""Weight-gradient products of the GPT-Neo-1.3B step (K = T = 131072 tokens, fp32 output) on hipBLASLt and on the
MFMA phase kernel (split-K into a workspace + deterministic reduce), in the layouts the step uses."""
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
    for I, O, lay in ((4096, 2048, "NT"), (2048, 4096, "NT"), (4096, 2048, "TN")):
        X = (torch.rand(T * I, device=dev) * 2 - 1).to(torch.bfloat16)
        dY = (torch.rand(T * O, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.zeros(I * O, device=dev)
        if lay == "NT":   # x transposed ([I][T]), dy as produced ([T][O])
            a, b = raw.Operand(X, 0, T), raw.Operand(dY, 1, O)
        else:             # x as produced ([T][I]), dy transposed ([O][T])
            a, b = raw.Operand(X, 1, I), raw.Operand(dY, 0, T)
        f = 2 * T * I * O / 1e12
        row = []
        for lt in (1, 0):
            raw.lt_set(bool(lt))
            t = timeit(lambda: raw.gemm(a, b, raw.Operand(C, 0, O), I, O, T))
            row.append(f"{'hipBLASLt' if lt else 'MFMA split-K'} {t * 1e3:.3f} ms ({f / t:.0f} TF/s)")
        raw.lt_set(True)
        print(f"dW [{I}][{O}] {lay}: " + " | ".join(row), flush=True)
        del X, dY, C


if __name__ == "__main__":
    main()
