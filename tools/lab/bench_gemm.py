#!/usr/bin/env python3
"""GEMM throughput on the model's shapes (GPT-Neo-1.3B, 32k tokens/GPU), random bf16 operands.
Interleaves repetitions so variants are compared in one process (cdna guide §5.4 rule 24)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

T = int(os.environ.get("T", 32768))
SHAPES = [  # (name, M, N, K, a_t, b_t, out_f32)
    ("fwd d->I", T, 4096, 2048, 0, 1, False), ("fwd I->d", T, 2048, 4096, 0, 1, False),
    ("dgrad I->d", T, 2048, 4096, 0, 0, False), ("dgrad d->I", T, 4096, 2048, 0, 0, False),
    ("wgrad d x I", 2048, 4096, T, 1, 1, True), ("wgrad I x d", 4096, 2048, T, 1, 1, True),
    ("logits fwd", T, 50304, 2048, 0, 1, False), ("logits dgrad", T, 2048, 50304, 0, 0, False),
    ("logits wgrad", 2048, 50304, T, 1, 1, True),
    ("wgradNT d x I", 2048, 4096, T, 0, 0, True), ("wgradNT I x d", 4096, 2048, T, 0, 0, True),
    ("sq8k NT", 8192, 8192, 8192, 0, 0, False), ("sq8k NN", 8192, 8192, 8192, 0, 1, False),
    ("sq8k TT f32", 8192, 8192, 8192, 1, 1, True), ("sq8k TN", 8192, 8192, 8192, 1, 0, False),
]


def main():
    dev = torch.device("cuda")
    bufs = {}
    for name, M, N, K, at, bt, f32 in SHAPES:
        A = torch.randn(M * K, device=dev).to(torch.bfloat16)
        B = torch.randn(N * K, device=dev).to(torch.bfloat16)
        C = torch.zeros(M * N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        bufs[name] = (A, B, C)
    res = {n: [] for n, *_ in SHAPES}
    for rep in range(5):
        for name, M, N, K, at, bt, f32 in SHAPES:
            A, B, C = bufs[name]
            ops = (raw.Operand(A, at, K if at == 0 else M), raw.Operand(B, bt, K if bt == 0 else N),
                   raw.Operand(C, 0, N))
            raw.gemm(*ops, M, N, K, beta=1.0 if f32 else 0.0)
            torch.cuda.synchronize()
            t = time.perf_counter()
            n = 3
            for _ in range(n):
                raw.gemm(*ops, M, N, K, beta=1.0 if f32 else 0.0)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / n
            res[name].append(2 * M * N * K / dt / 1e12)
    tag = os.environ.get("OBST_GEMM_BIG", "2") + "/ks" + os.environ.get("OBST_GEMM_KSPLIT", "1")
    for name, *_ in SHAPES:
        v = sorted(res[name])
        print(f"[big={tag}] {name:14s} median {v[len(v) // 2]:7.1f} TFLOP/s  max {v[-1]:7.1f}")


if __name__ == "__main__":
    main()
