#!/usr/bin/env python3
"""Plain PyTorch-ROCm eager baseline of the GPT-Neo-1.3B-shaped model (BASELINE.md "comparison baseline 1"):
the same layer shapes as `configs/gpt_neo_1.3b.json` built from stock torch modules -- factorised input embedding
(vocab x 512 gather, 512 -> 2048 linear), 24 x [LayerNorm -> 2048 -> 4096 linear -> k, q, v (4096 -> 2048 each) ->
causal SDPA (16 heads x 128) -> + residual; LayerNorm -> 2048 -> 4096 gelu(tanh) -> 4096 -> 2048 -> + residual],
2048 -> vocab output projection, softmax cross-entropy. bf16 autocast over fp32 parameters, fused AdamW (torch has
no SM3), synthetic tokens. Prints one line: tokens/s, ms/step, peak memory.

    python tools/torch_baseline.py [--batch 16] [--steps 6] [--warmup 3] [--compile 0]
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

V, D, H, DH, L, S, FF, E = 50257, 2048, 16, 128, 24, 2048, 4096, 512


class Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.n1, self.n2 = nn.LayerNorm(D), nn.LayerNorm(D)
        self.w_in = nn.Linear(D, FF, bias=False)
        self.wk, self.wq, self.wv = (nn.Linear(FF, D, bias=False) for _ in range(3))
        self.f1, self.f2 = nn.Linear(D, FF, bias=False), nn.Linear(FF, D, bias=False)

    def forward(self, x):
        b, s, _ = x.shape
        base = self.w_in(self.n1(x))
        k, q, v = (w(base).view(b, s, H, DH).transpose(1, 2) for w in (self.wk, self.wq, self.wv))
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        x = x + o.transpose(1, 2).reshape(b, s, D)
        return x + self.f2(F.gelu(self.f1(self.n2(x)), approximate="tanh"))


class Model(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(V, E)
        self.inp = nn.Linear(E, D, bias=False)
        self.blocks = nn.ModuleList(Block() for _ in range(L))
        self.out = nn.Linear(D, V, bias=False)

    def forward(self, x, y):
        h = self.inp(self.emb(x))
        for blk in self.blocks:
            h = blk(h)
        logits = self.out(h)
        return F.cross_entropy(logits.float().view(-1, V), y.view(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--compile", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = Model().to(dev)
    nparams = sum(p.numel() for p in model.parameters())
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, fused=True)
    fwd = torch.compile(model) if args.compile else model
    g = torch.Generator(device=dev).manual_seed(1)
    toks = torch.randint(0, V, (args.batch, S + 1), device=dev, generator=g)
    x, y = toks[:, :-1].contiguous(), toks[:, 1:].contiguous()

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = fwd(x, y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"baseline": "torch eager" + (" + compile" if args.compile else ""), "params": nparams,
                      "batch": args.batch, "seq": S, "tokens_per_s": round(args.batch * S / dt, 1),
                      "ms_per_step": round(dt * 1e3, 2), "loss": round(float(loss), 4),
                      "peak_gib": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)}), flush=True)


if __name__ == "__main__":
    main()
