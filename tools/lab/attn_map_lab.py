"""Attention-map kernels at the kbench shape (B16 S2048 H16 D128 causal): forward with / without the bias map and the
backward, a few reps each, for `rocprofv3 --kernel-trace --stats` (per-kernel split: forward, dq, dk/dv, fold)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

B, S, H, D = 16, 2048, 16, 128
dev = torch.device("cuda")
BF = torch.bfloat16
q, k, v, do = ((torch.randn(B, S, H, D, device=dev) * 0.5).to(BF) for _ in range(4))
bias = torch.randn(H, S, S, device=dev) * 0.1
o = torch.empty_like(q)
lse = torch.empty(B * H * S, device=dev)
dq, dk, dv = (torch.empty_like(q) for _ in range(3))
delta = torch.empty_like(lse)
db = torch.empty(H, S, S, device=dev)
bs = raw.attn_map_bsplit(B, S, H)
pb = torch.zeros(bs, H, S, S, device=dev) if bs > 1 else None
sc = D ** -0.5
unit = B * H * S * S / 2 * D * 2


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


f0 = t(lambda: raw.attn_map_fwd(q, k, v, o, lse, None, None, B, S, H, D, sc, True))
f1 = t(lambda: raw.attn_map_fwd(q, k, v, o, lse, bias, None, B, S, H, D, sc, True))


def bwd():
    if pb is not None:
        pb.zero_()
    raw.attn_map_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, bias, None, db, None, B, S, H, D, sc, True, pb)


b1 = t(bwd)
print(f"fwd no-map {f0:.1f} us ({2 * unit / f0 / 1e9:.3f} PF/s), fwd bias {f1:.1f} us ({2 * unit / f1 / 1e9:.3f}), "
      f"bwd bias {b1:.1f} us ({5 * unit / b1 / 1e9:.3f}), bsplit {bs}", flush=True)
