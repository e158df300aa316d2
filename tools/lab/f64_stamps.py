#!/usr/bin/env python3
"""Per-block cycle stamps of the 64-query forward built with FWD64_DBG & 64 (OBST_KERNELS=<variant .so>,
OBST_ATTN_IMPL=3): prologue / steps / epilogue cycles per block, cycles per step."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402


def main():
    B, S, H, D = int(os.environ.get("B", 64)), 2048, 16, 128
    causal = os.environ.get("CAUSAL", "1") == "1"
    dev = torch.device("cuda")
    ld = 3 * H * D
    buf = (torch.randn(B * S * ld, device=dev) * 0.5).to(torch.bfloat16)
    k, q, v = (buf[j * H * D:] for j in range(3))
    o = torch.empty(B * S * H * D, device=dev, dtype=torch.bfloat16)
    lse = torch.zeros(B * H * S, device=dev)
    for _ in range(3):
        raw.attn_fwd(q, k, v, o, lse, B, S, H, D, ld, D ** -0.5, causal, ld_o=H * D)
    torch.cuda.synchronize()
    nblk = (S + 255) // 256 * B * H
    st = lse[:4 * nblk].view(nblk, 4).cpu().numpy().astype(np.float64)
    pro, steps, epi, n = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    print(f"causal={causal} B={B}: blocks {nblk}; prologue {pro.mean():.0f} cyc, steps {steps.mean():.0f} cyc "
          f"({(steps / n).mean():.0f} per step, {n.mean():.1f} steps), epilogue {epi.mean():.0f} cyc; "
          f"per-step p10/p50/p90 {np.percentile(steps / n, 10):.0f}/{np.percentile(steps / n, 50):.0f}/"
          f"{np.percentile(steps / n, 90):.0f}")


if __name__ == "__main__":
    main()
