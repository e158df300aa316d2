#!/usr/bin/env python3
"""GPT-Neo-1.3B step shapes (T = 131072 tokens) on the hand-written MFMA GEMM (csrc/kernels/gemm.hip) against
hipBLASLt: plain products, and the activation GEMMs (gelu with the pre-activation side output; gelu backward) as
one fused MFMA launch vs hipBLASLt + the elementwise kernel."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 131072))
SHAPES = [(T, 4096, 2048), (T, 2048, 4096), (T, 6144, 4096), (T, 4096, 6144)]


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
    for M, N, K in SHAPES:
        A = (torch.rand(M * K, device=dev) * 2 - 1).to(torch.bfloat16)
        Bw = (torch.rand(N * K, device=dev) * 2 - 1).to(torch.bfloat16)     # [N][K] (K-contiguous weight copy)
        C = torch.empty(M * N, device=dev, dtype=torch.bfloat16)
        Z = torch.empty(M * N, device=dev, dtype=torch.bfloat16)
        ops = (raw.Operand(A, 0, K), raw.Operand(Bw, 0, K), raw.Operand(C, 0, N))
        f = 2 * M * N * K / 1e12
        row = []
        for lt in (2, 1, 0):     # 2: hipBLASLt's own GELU_AUX / DGELU epilogues (tanh-form gelu, as the reference)
            raw.lt_set(bool(lt))
            if lt == 2:
                raw.L.lib().obst_blaslt_set(2)
                raw._LT = 2
            tp = timeit(lambda: raw.gemm(*ops, M, N, K))
            ta = timeit(lambda: raw.gemm(*ops, M, N, K, act="gelu", Zout=Z))
            tb = timeit(lambda: raw.gemm(*ops, M, N, K, act="gelu", act_bwd=True, Zin=Z))
            row.append(f"{['MFMA', 'hipBLASLt', 'hipBLASLt-epilogue'][lt]}: plain {tp * 1e3:.3f} ms ({f / tp:.0f} TF/s) "
                       f"gelu+Zout {ta * 1e3:.3f} ms gelu-bwd {tb * 1e3:.3f} ms")
        raw.lt_set(True)
        print(f"M {M} N {N} K {K} | " + " | ".join(row), flush=True)
        del A, Bw, C, Z


if __name__ == "__main__":
    main()
