"""Skinny-M (decode-step) GEMM: csrc/kernels/skinny.hip vs hipBLASLt (both weight layouts), graph-replayed per-call
time over the GPT-Neo-1.3B decode shapes (weights L2/MALL-warm: replayed back to back).
    python tools/bench_skinny.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def run(M, K, N, skinny, kcontig, iters=200):
    raw._SKINNY = skinny
    a = torch.randn(M * K, device="cuda").bfloat16()
    w = torch.randn(K * N, device="cuda").bfloat16()
    bop = raw.Operand(w, 0, K) if kcontig else raw.Operand(w, 1, N)   # [N][K] copy or the stored [K][N]
    c = torch.empty(M * N, device="cuda", dtype=torch.bfloat16)
    f = lambda: raw.gemm(raw.Operand(a, 0, K), bop, raw.Operand(c, 0, N), M, N, K)  # noqa: E731
    for _ in range(10):
        f()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters // 20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    return us, K * N * 2 / us / 1e3


for M, K, N in [(32, 2048, 2048), (32, 4096, 2048), (32, 2048, 4096), (32, 2048, 6144), (32, 2048, 8192),
                (32, 8192, 2048), (16, 2048, 2048), (32, 2048, 50304)]:
    ul, bl = run(M, K, N, False, False)
    ut, bt = run(M, K, N, False, True)
    us, bs = run(M, K, N, True, True)
    print(f"M{M} K{K} N{N}: hipBLASLt [K][N] {ul:7.1f} us ({bl:5.0f} GB/s)  hipBLASLt [N][K] {ut:7.1f} us "
          f"({bt:5.0f} GB/s)  MFMA skinny {us:7.1f} us ({bs:5.0f} GB/s)", flush=True)
