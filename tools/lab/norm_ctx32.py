"""ctx32_mixer's norm passes at their step shapes (tokens 256 x 2048, 8 heads): per kernel us and GB/s moved.

  F 256 (features_per_head, group): forward, forward + gelu, backward + bf16 stream gradient + parameters,
        backward through gelu + parameters
  F 512 (the bottleneck's mid, group): forward, backward through relu (in_relu) + parameters

OBST_KERNELS=<variant .so> selects a build variant (A/B in one process list: tools/lab/norm_ab.sh).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

BF = torch.bfloat16


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ts = []
    for i in range(reps):
        ev[i].record()
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    for i in range(reps):
        ts.append(ev[i].elapsed_time(ev[i + 1]) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=256 * 2048)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("OBST_KERNELS", "tree")))
    args = ap.parse_args()
    dev = torch.device("cuda")
    H = args.heads
    out = {"tag": args.tag}
    for F in (256, 512):
        rows = args.tokens * H
        n = rows * F
        torch.manual_seed(0)
        x = (torch.randn(n, device=dev) * 2).to(BF)
        dy = torch.randn(n, device=dev).to(BF)
        r = torch.randn(n, device=dev).to(BF)
        sc = torch.randn(H * F, device=dev) * 0.1 + 1
        sh = torch.randn(H * F, device=dev) * 0.1
        y, dx = torch.empty_like(x), torch.empty_like(x)
        stats = torch.empty(2 * rows, device=dev)
        dsc, dsh = torch.zeros(H * F, device=dev), torch.zeros(H * F, device=dev)
        gb = lambda b, us: round(b * n / us / 1e3, 1)   # noqa: E731
        if F == 256:   # the streaming reference: torch's bf16 copy of the same bytes
            us = timed(lambda: y.copy_(x), args.reps)
            out["copy256"] = (round(us, 1), gb(4, us))
        us = timed(lambda: raw.norm_fwd(x, sc, sh, y, stats, rows, F, H), args.reps)
        out[f"fwd{F}"] = (round(us, 1), gb(4, us))
        if F == 256:
            us = timed(lambda: raw.norm_fwd(x, sc, sh, y, stats, rows, F, H, act="gelu"), args.reps)
            out[f"fwd_gelu{F}"] = (round(us, 1), gb(4, us))
            raw.norm_fwd(x, sc, sh, y, stats, rows, F, H)
            us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, dsc, dsh, rows, F, H, F, R=r), args.reps)
            out[f"bwd_R{F}"] = (round(us, 1), gb(8, us))
            us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, dsc, dsh, rows, F, H, F, shift=sh, act="gelu"),
                       args.reps)
            out[f"bwd_gelu{F}"] = (round(us, 1), gb(6, us))
        else:
            raw.norm_fwd(x, sc, sh, y, stats, rows, F, H)
            us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, dsc, dsh, rows, F, H, F, in_relu=True),
                       args.reps)
            out[f"bwd_relu{F}"] = (round(us, 1), gb(6, us))
        del x, dy, r, y, dx
        torch.cuda.empty_cache()
    # GPT-Neo-1.3B's norms (64 x 2048 tokens, 2048 features, one group): forward, backward + residual + parameters
    rows, F = 64 * 2048, 2048
    n = rows * F
    x = (torch.randn(n, device=dev) * 2).to(BF)
    dy, r = torch.randn(n, device=dev).to(BF), torch.randn(n, device=dev).to(BF)
    sc, sh = torch.randn(F, device=dev) * 0.1 + 1, torch.randn(F, device=dev) * 0.1
    y, dx = torch.empty_like(x), torch.empty_like(x)
    stats = torch.empty(2 * rows, device=dev)
    dsc, dsh = torch.zeros(F, device=dev), torch.zeros(F, device=dev)
    us = timed(lambda: raw.norm_fwd(x, sc, sh, y, stats, rows, F, 1), args.reps)
    out["neo_fwd"] = (round(us, 1), round(4 * n / us / 1e3, 1))
    us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, dsc, dsh, rows, F, 1, F, R=r), args.reps)
    out["neo_bwd_R"] = (round(us, 1), round(8 * n / us / 1e3, 1))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
