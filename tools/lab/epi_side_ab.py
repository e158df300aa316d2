"""What the side-input epilogues cost on GPT-Neo-1.3B's step shapes: the same product plain, with the bf16 residual
(R, the block output projections) and with the gelu backward (act_bwd + Zin, the FFN-in dgrad). B stored [N][K]
(K-contiguous: the row-layout epilogue) as the model's weights are. Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

BF = torch.bfloat16


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    for i in range(reps):
        ev[i].record()
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(reps))
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    tag = os.path.basename(os.environ.get("OBST_KERNELS", "tree"))
    for name, M, N, K in (("4d->d (+R)", 131072, 2048, 8192), ("d->d (+R)", 131072, 2048, 2048),
                          ("dgrad d->4d (gelu')", 131072, 8192, 2048)):
        a = (torch.randn(M, K, device=dev) * 0.1).to(BF)
        b = (torch.randn(N, K, device=dev) * 0.1).to(BF)   # [N][K]
        c = torch.empty(M, N, device=dev, dtype=BF)
        side = torch.randn(M, N, device=dev).to(BF)
        A, B, C = raw.Operand(a, 0, K), raw.Operand(b, 1, K), raw.Operand(c, 0, N)
        plain = timed(lambda: raw.gemm(A, raw.Operand(b, 0, K), C, M, N, K))
        if "gelu" in name:
            us = timed(lambda: raw.gemm(A, raw.Operand(b, 0, K), C, M, N, K, act="gelu", act_bwd=True, Zin=side))
        else:
            us = timed(lambda: raw.gemm(A, raw.Operand(b, 0, K), C, M, N, K, R=side))
        print(json.dumps({"tag": tag, "shape": name, "us_plain": round(plain, 1), "us_side": round(us, 1),
                          "side_cost": round(us / plain - 1, 4)}), flush=True)
        del a, b, c, side
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
