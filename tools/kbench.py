#!/usr/bin/env python3
"""Maintained kernel harness: the training step's hot kernels at their GPT-Neo-1.3B shapes, one JSON line each.

  python tools/kbench.py [gemm|attn|attn_map|norm|ew|all] [--reps N] [--tokens T] [--check profiles/kbench_floor.json]

* gemm      -- every plain product of the step (fwd / dgrad / fp32 wgrad / logits) on hipBLASLt and on the
               hand-written gemm4w kernel, interleaved in one process (cdna guide §5.4 rule 24): TF/s and ratio.
               The per-tile clock breakdown of gemm4w lives in the C++ harness (tools/gemm_bench.cpp, STAMPS=1).
* attn      -- flash attention fwd / bwd (B, S 2048, H 16, D 128, causal, interleaved k|q|v as in the step):
               effective causal PF/s (fwd 2 units, bwd 5 units of B*H*S*S/2*D*2 FLOPs).
* attn_map  -- the biased_softmax / scale_attention_map kernels (csrc/kernels/attn_map.hip) at the same shape.
* norm      -- norm fwd / bwd (+ residual gradient, + parameter gradients): GB/s of the bytes each must move.
* ew        -- the streaming elementwise kernels (gelu fwd / bwd, add): GB/s.

--check FLOOR.json (the perf-regression gate of tools/gpu_final.sh): every emitted line whose key (kernel, shape) has
floors in the file must reach each floored metric within --tol (default 5 %); the exit status is 1 otherwise.

The profiles under profiles/ quote these numbers; the one-off A/B scripts next to it (bench_*.py, gpu_*.sh) are the
lab notes behind individual measurements (tools/README.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

BF = torch.bfloat16


def timed(fn, reps: int) -> float:
    """mean microseconds per call over `reps` calls after two warm-up calls"""
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


EMITTED = []


def emit(**kw):
    EMITTED.append(kw)
    print(json.dumps(kw), flush=True)


def line_key(row: dict) -> str:
    return row["kernel"] + (f" {row['shape']}" if "shape" in row else "")


def section_of(key: str) -> str:
    """the kbench section (command-line `what`) that emits a floor key"""
    if key.startswith("gemm"):
        return "gemm"
    if key.startswith("mixer"):
        return "mixer"
    if key.startswith("attention_map"):
        return "attn_map"
    if key.startswith("attention"):
        return "attn"
    if key.startswith("norm"):
        return "norm"
    return "ew"


def missing(floors: dict, seen: set, sections) -> list:
    """floor keys of the sections that ran but that no emitted row carries (a renamed / dropped kernel or shape
    must not silently skip its floor)"""
    return sorted(k for k in floors if section_of(k) in sections and k not in seen)


def check(rows, floors: dict, tol: float = 0.05):
    """-> list of (key, metric, value, floor) for every floored metric below floor * (1 - tol); higher is better for
    every metric in the floor file (TF/s, PF/s, GB/s)"""
    bad = []
    for row in rows:
        for metric, floor in floors.get(line_key(row), {}).items():
            v = row.get(metric)
            if v is None or v < floor * (1.0 - tol):
                bad.append((line_key(row), metric, v, floor))
    return bad


def bench_gemm(T: int, reps: int):
    d, i4, V = 2048, 8192, 50304
    shapes = [  # name, M, N, K, a_t, b_t, out_f32 (layouts as the step issues them)
        ("fwd d->4d", T, i4, d, 0, 0, False), ("fwd 4d->d", T, d, i4, 0, 0, False),
        ("fwd kqv d->3d", T, 3 * d, d, 0, 0, False), ("dgrad 3d->d", T, d, 3 * d, 0, 0, False),
        ("logits", T, V, d, 0, 0, False), ("logits dgrad", T, d, V, 0, 0, False),
        ("wgrad d x 4d", d, i4, T, 1, 1, True), ("wgrad 4d x d", i4, d, T, 1, 1, True),
        ("wgrad logits", d, V, T, 0, 1, True),
    ]
    dev = torch.device("cuda")
    for name, M, N, K, at, bt, f32 in shapes:
        A = (torch.randn(M * K, device=dev) * 0.5).to(BF)
        B = (torch.randn(N * K, device=dev) * 0.5).to(BF)
        C = torch.zeros(M * N, device=dev, dtype=torch.float32 if f32 else BF)
        ops = (raw.Operand(A, at, K if at == 0 else M), raw.Operand(B, bt, K if bt == 0 else N), raw.Operand(C, 0, N))
        t = {}
        for rnd in range(2):   # interleaved: library, hand-written, library, hand-written
            for lt in (1, 0):
                old = raw.lt_set(lt)
                us = timed(lambda: raw.gemm(*ops, M, N, K), reps)
                raw.lt_set(old)
                t[lt] = min(t.get(lt, 1e30), us)
        fl = 2.0 * M * N * K
        emit(kernel="gemm", shape=name, M=M, N=N, K=K, a_t=at, b_t=bt, out_f32=f32,
             us_hipblaslt=round(t[1], 1), us_gemm4w=round(t[0], 1), tflops_hipblaslt=round(fl / t[1] / 1e6, 1),
             tflops_gemm4w=round(fl / t[0] / 1e6, 1), gemm4w_over_hipblaslt=round(t[1] / t[0], 3))
        del A, B, C


def bench_mixer(reps: int):
    """the learned token mixer's GEMMs (K03, ctx32_mixer: 32 x 2048 tokens, 8 heads x 256): y = tril(W) x
    (tri 1) and dx = tril(W)^T dy (tri 2) on gemm4w against the persistent phase kernel (OBST_GEMM_4W=0 path);
    effective TF/s count only the causal half"""
    import ctypes
    from homebrewnlp_mtf_amd.ops import _lib as L
    B, S, H, Fd = 32, 2048, 8, 256
    dev = torch.device("cuda")
    x = (torch.randn(B * S * H * Fd, device=dev) * 0.5).to(BF)
    w = torch.tril((torch.randn(H, S, S, device=dev) * 0.05)).to(BF).reshape(-1)
    y = torch.empty_like(x)
    hf = H * Fd
    fl = B * H * S * S * Fd   # 2 * S * S / 2 per (batch, head, feature)
    for name, a_t, tri in (("mixer y=tril(W)x", 0, 1), ("mixer dx=tril(W)^T dy", 1, 2)):
        def run():
            raw.gemm(raw.Operand(w, a_t, S, 0, S * S), raw.Operand(x, 1, hf, S * hf, Fd),
                     raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=tri)
        t = {}
        for rnd in range(2):
            for on in (0, 1):
                old = L.lib().obst_gemm4w_set(on)
                t[on] = min(t.get(on, 1e30), timed(run, reps))
                L.lib().obst_gemm4w_set(old)
        emit(kernel="gemm", shape=name, us_phase=round(t[0], 1), us_gemm4w=round(t[1], 1),
             tflops_phase=round(fl / t[0] / 1e6, 1), tflops_gemm4w=round(fl / t[1] / 1e6, 1),
             gemm4w_over_phase=round(t[0] / t[1], 3))


def _qkv(B, S, H, D, dev):
    ld = 3 * H * D
    buf = (torch.randn(B * S * ld, device=dev) * 0.5).to(BF)
    return buf, ld


def bench_attn(B: int, reps: int):
    S, H, D = 2048, 16, 128
    dev = torch.device("cuda")
    buf, ld = _qkv(B, S, H, D, dev)
    gbuf = torch.empty_like(buf)
    k, q, v = (buf[j * H * D:] for j in range(3))
    dk, dq, dv = (gbuf[j * H * D:] for j in range(3))
    o = torch.empty(B * S * H * D, device=dev, dtype=BF)
    do = (torch.randn(B * S * H * D, device=dev) * 0.5).to(BF)
    lse = torch.empty(B * H * S, device=dev)
    delta = torch.empty_like(lse)
    sc = D ** -0.5
    unit = B * H * S * S / 2 * D * 2
    f = timed(lambda: raw.attn_fwd(q, k, v, o, lse, B, S, H, D, ld, sc, True, ld_o=H * D), reps)
    b = timed(lambda: raw.attn_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, H, D, ld, sc, True, ld_o=H * D),
              reps)
    emit(kernel="attention", B=B, S=S, H=H, D=D, causal=True, us_fwd=round(f, 1), us_bwd=round(b, 1),
         pflops_fwd=round(2 * unit / f / 1e9, 3), pflops_bwd=round(5 * unit / b / 1e9, 3))


def bench_attn_map(B: int, reps: int):
    S, H, D = 2048, 16, 128
    dev = torch.device("cuda")
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
    f = timed(lambda: raw.attn_map_fwd(q, k, v, o, lse, bias, None, B, S, H, D, sc, True), reps)

    def bwd():
        if pb is not None:
            pb.zero_()
        raw.attn_map_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, bias, None, db, None, B, S, H, D, sc, True, pb)
    b = timed(bwd, reps)
    emit(kernel="attention_map(biased_softmax)", B=B, S=S, H=H, D=D, causal=True, us_fwd=round(f, 1),
         us_bwd=round(b, 1), pflops_fwd=round(2 * unit / f / 1e9, 3), pflops_bwd=round(5 * unit / b / 1e9, 3),
         bias_grad_slices=bs)


def bench_norm(T: int, reps: int):
    F = 2048
    dev = torch.device("cuda")
    x = (torch.randn(T * F, device=dev) * 2).to(BF)
    dy, r = ((torch.randn(T * F, device=dev)).to(BF) for _ in range(2))
    sc, sh = torch.ones(F, device=dev), torch.zeros(F, device=dev)
    y, dx = torch.empty_like(x), torch.empty_like(x)
    stats = torch.empty(2 * T, device=dev)
    dsc, dsh = torch.zeros(F, device=dev), torch.zeros(F, device=dev)
    us = timed(lambda: raw.norm_fwd(x, sc, sh, y, stats, T, F, 1), reps)
    emit(kernel="norm_fwd", rows=T, F=F, us=round(us, 1), gbps=round(2 * T * F * 2 / us / 1e3, 1))
    for name, R, params in (("norm_bwd+R+params", r, True), ("norm_bwd+R", r, False), ("norm_bwd", None, False)):
        args = (dsc, dsh) if params else (None, None)
        us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, args[0], args[1], T, F, 1, F, R=R), reps)
        nbytes = (3 + (1 if R is not None else 0)) * T * F * 2
        emit(kernel=name, rows=T, F=F, us=round(us, 1), gbps=round(nbytes / us / 1e3, 1))


def bench_ew(T: int, reps: int):
    n = T * 8192
    dev = torch.device("cuda")
    x, z = ((torch.randn(n, device=dev)).to(BF) for _ in range(2))
    y = torch.empty_like(x)
    for name, fn, streams in (("gelu_fwd", lambda: raw.elementwise("act", x, y, act="gelu"), 2),
                              ("gelu_bwd", lambda: raw.elementwise("act_bwd", x, y, z=z, act="gelu"), 3),
                              ("add", lambda: raw.elementwise("add", x, y, z=z), 3)):
        us = timed(fn, reps)
        emit(kernel=name, elements=n, us=round(us, 1), gbps=round(streams * n * 2 / us / 1e3, 1))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all", choices=["gemm", "mixer", "attn", "attn_map", "norm", "ew", "all"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=131072, help="tokens per step (GPT-Neo-1.3B: 64 x 2048)")
    ap.add_argument("--batch", type=int, default=64, help="attention batch at S 2048")
    ap.add_argument("--check", default=None, help="floor file: fail on a regression past --tol")
    ap.add_argument("--tol", type=float, default=0.05)
    a = ap.parse_args(argv)
    todo = ["gemm", "mixer", "attn", "attn_map", "norm", "ew"] if a.what == "all" else [a.what]
    for w in todo:
        if w == "gemm":
            bench_gemm(a.tokens, a.reps)
        elif w == "mixer":
            bench_mixer(a.reps)
        elif w == "attn":
            bench_attn(a.batch, a.reps)
        elif w == "attn_map":
            bench_attn_map(min(a.batch, 16), a.reps)
        elif w == "norm":
            bench_norm(a.tokens, a.reps)
        else:
            bench_ew(a.tokens, a.reps)
    if a.check:
        with open(a.check) as f:
            floors = json.load(f)["floors"]
        bad = check(EMITTED, floors, a.tol)
        seen = {line_key(r) for r in EMITTED}
        for key, metric, v, floor in bad:
            print(f"REGRESSION {key}: {metric} {v} < floor {floor} - {a.tol:.0%}", flush=True)
        gone = missing(floors, seen, todo)
        for key in gone:
            print(f"MISSING {key}: floored but not emitted by its section", flush=True)
        n = sum(len(m) for k, m in floors.items() if k in seen)
        print(f"kbench check: {n - len(bad)}/{n} floored metrics pass, {len(gone)} floored keys missing", flush=True)
        if bad or gone:
            sys.exit(1)


if __name__ == "__main__":
    main()
