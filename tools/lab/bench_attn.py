#!/usr/bin/env python3
"""Flash-attention kernel throughput on the GPT-Neo-1.3B shape (B16 S2048 H16 D128, causal), bf16 random data.
FLOP convention: one "unit" = B*H*S*S/2*D*2 (a causal S x S x D product); fwd = 2 units, bwd = 5 units (dK/dV
kernel recomputes S and dP: 4, dQ kernel recomputes S and dP: 3 -> 7 executed, 5 useful)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def main():
    B, S, H, D = (int(os.environ.get(k, v)) for k, v in (("B", 16), ("S", 2048), ("H", 16), ("D", 128)))
    causal = os.environ.get("CAUSAL", "1") == "1"
    dev = torch.device("cuda")
    # KQV=1: q, k, v (and dq, dk, dv) as column slices of one interleaved k|q|v buffer [B*S][3*H*D], the layout of
    # the training step's fused projection (row stride 3*H*D); o / do stay [B*S][H*D]
    kqv = os.environ.get("KQV", "0") == "1"
    ld = (3 if kqv else 1) * H * D
    mk = lambda n: (torch.randn(n, device=dev) * 0.5).to(torch.bfloat16)  # noqa: E731
    if kqv:
        buf, gbuf = mk(B * S * ld), torch.empty(B * S * ld, device=dev, dtype=torch.bfloat16)
        k, q, v = (buf[j * H * D:] for j in range(3))
        dk, dq, dv = (gbuf[j * H * D:] for j in range(3))
        do = mk(B * S * H * D)
    else:
        q, k, v, do = (mk(B * S * ld) for _ in range(4))
        dq, dk, dv = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    o = torch.empty_like(do)
    lse = torch.empty(B * H * S, device=dev)
    delta = torch.empty(B * H * S, device=dev)
    scale = D ** -0.5
    unit = B * H * S * S * D * (1.0 if causal else 2.0)
    # RES=1: the forward epilogue also writes bf16(o) + residual (the training step's fused residual add)
    res_t = mk(B * S * H * D) if os.environ.get("RES", "0") == "1" else None
    out_t = torch.empty_like(res_t) if res_t is not None else None
    fwd = lambda: raw.attn_fwd(q, k, v, o, lse, B, S, H, D, ld, scale, causal, ld_o=H * D,  # noqa: E731
                               residual=res_t, out=out_t)
    bwd = lambda: raw.attn_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, H, D, ld, scale, causal,  # noqa: E731
                               ld_o=H * D)
    res = {"fwd": [], "bwd": []}
    for rep in range(5):
        only = os.environ.get("ONLY", "")
        for name, fn, units in (("fwd", fwd, 2), ("bwd", bwd, 5)):
            if only and name != only:
                continue
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            n = 5
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / n
            res[name].append((dt * 1e3, units * unit / dt / 1e12))
    for name, v in res.items():
        if not v:
            continue
        v.sort()
        ms, tf = v[len(v) // 2]
        print(f"attn {name} B{B} S{S} H{H} D{D} causal={causal} kqv={int(kqv)} res={int(res_t is not None)}: {ms:.3f} ms  {tf:.0f} TFLOP/s (useful)")


if __name__ == "__main__":
    main()
