#!/usr/bin/env python3
"""Maintained kernel harness: the training step's hot kernels at their GPT-Neo-1.3B shapes, one JSON line each.

  python tools/kbench.py [gemm|attn|attn_map|norm|ew|all] [--reps N] [--tokens T] [--check profiles/kbench_floor.json]

* gemm      -- every plain product of the step (fwd / dgrad / fp32 wgrad / logits) on the hand-written gemm4w
               kernel: TF/s (the hipBLASLt A/B lives in tools/lab/g4w_sched.cpp; no library GEMM is linked).
               The per-tile clock breakdown of gemm4w lives in the C++ harness (tools/gemm_bench.cpp, STAMPS=1).
* attn      -- flash attention fwd / bwd (B, S 2048, H 16, D 128, causal, interleaved k|q|v as in the step):
               effective causal PF/s (fwd 2 units, bwd 5 units of B*H*S*S/2*D*2 FLOPs).
* attn_map  -- biased_softmax at the same shape: the flash kernels with the map hook (attention.hip) by default,
               the attn_map.hip kernels with OBST_MAP_FLASH=0.
* norm      -- norm fwd / bwd (+ residual gradient, + parameter gradients): GB/s of the bytes each must move.
* ew        -- the streaming elementwise kernels (gelu fwd / bwd, add): GB/s.
* gate      -- one row per hot-kernel family (GATE), each between its own two calibrations: the perf gate that
               tests/test_gpu_perf_gate.py runs inside `pytest -m gpu`.

Timing: every number is the MEDIAN of --reps (default 20) individually timed calls after two warm-up calls; where
two implementations are compared their samples are interleaved call by call (cdna guide §5.4 rule 24).

Calibration (same process): a bare bf16 MFMA loop on random register operands (csrc/kernels/calib.hip; TF/s) and a
512 MiB device copy (GB/s), measured before and after each section. Every emitted line carries the two and the
ratio of each metric to its calibration (``ratio_<metric>``): compute metrics (TF/s, PF/s) over the MFMA loop, memory
metrics (GB/s) over the copy. Devices differ by up to ~12 % on an MFMA loop at the same code (MI355X_MICROARCH.md,
'DVFS give-back' item 5), so the gate compares ratios.

--check FLOOR.json (the perf-regression gate of tools/gpu_final.sh): every emitted line whose key (kernel, shape) has
floors in the file must reach, within --tol (default 3 %), its floored calibration ratio (``ratios``) OR its absolute
floor (``floors``) -- a metric regresses only when it misses both (check_either) -- and every floored key of a
section that ran must have been emitted; the exit status is 1 otherwise. --write-floors PATH writes the observed ratios as a new floor file.

The profiles under profiles/ quote these numbers; the one-off A/B scripts next to it (bench_*.py, gpu_*.sh) are the
lab notes behind individual measurements (tools/README.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import typing

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402

BF = torch.bfloat16


def timed_many(fns, reps: int):
    """median microseconds per call of each fn: `reps` samples, the fns interleaved call by call, every call timed
    by its own pair of events (after two warm-up calls each)"""
    for fn in fns:
        for _ in range(2):
            fn()
    torch.cuda.synchronize()
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
           for _ in fns]
    for r in range(reps):
        for i, fn in enumerate(fns):
            evs[i][r][0].record()
            fn()
            evs[i][r][1].record()
    torch.cuda.synchronize()
    out = []
    for i in range(len(fns)):
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in evs[i])
        out.append(t[len(t) // 2])
    return out


def timed(fn, reps: int) -> float:
    """median microseconds per call over `reps` individually timed calls after two warm-up calls"""
    return timed_many([fn], reps)[0]


CALIB = {}


def calibrate(reps: int = 20):
    """same-process calibration: bf16 MFMA loop TF/s (csrc/kernels/calib.hip) and a 512 MiB device copy GB/s"""
    from homebrewnlp_mtf_amd.ops import _lib as L
    dev = torch.device("cuda")
    sink = torch.empty(2048 * 256, device=dev)
    iters = 1024
    fl = float(L.lib().obst_calib_mfma_flops(iters))
    us = timed(lambda: L.check(L.lib().obst_calib_mfma(sink.data_ptr(), iters, L.stream_ptr()), "calib"), reps)
    src = torch.randn(128 * 2 ** 20, device=dev)
    dst = torch.empty_like(src)
    cus = timed(lambda: dst.copy_(src), reps)
    return {"mfma_tflops": fl / us / 1e6, "copy_gbps": 2 * src.numel() * 4 / cus / 1e3}


def section_calib(before: dict, after: dict) -> dict:
    return {k: (before[k] + after[k]) / 2 for k in before}


EMITTED = []
PENDING = []


def emit(**kw):
    """queue a row; flush_rows() attaches the section's calibration and ratios and prints it"""
    PENDING.append(kw)


def metric_kind(metric: str) -> str:
    return "copy_gbps" if metric.startswith("gbps") else "mfma_tflops"


def metric_scale(metric: str) -> float:
    """to TF/s (compute) or GB/s (memory)"""
    return 1000.0 if metric.startswith("pflops") else 1.0


def flush_rows(cal: dict):
    for kw in PENDING:
        kw["calib_mfma_tflops"] = round(cal["mfma_tflops"], 1)
        kw["calib_copy_gbps"] = round(cal["copy_gbps"], 1)
        for m in [k for k in kw if k.startswith(("tflops", "pflops", "gbps")) and isinstance(kw[k], (int, float))]:
            kw["ratio_" + m] = round(kw[m] * metric_scale(m) / cal[metric_kind(m)], 4)
        EMITTED.append(kw)
        print(json.dumps(kw), flush=True)
    PENDING.clear()


def line_key(row: dict) -> str:
    return row["kernel"] + (f" {row['shape']}" if "shape" in row else "")


def section_of(key: str) -> str:
    """the kbench section (command-line `what`) that emits a floor key"""
    if key.startswith(("mixer", "gemm mixer")):
        return "mixer"
    if key.startswith("gemm"):
        return "gemm"
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


def check_either(rows, floors: dict, tol: float = 0.03, ratios: typing.Optional[dict] = None):
    """the gate's rule: a metric regresses only when it misses BOTH its calibration-ratio floor and its absolute
    floor. The same-process calibrations themselves move between boxes (MFMA loop 1904-2091 TF/s, device copy
    4.6-5.3 TB/s in rounds 5-6) while the kernels' own numbers do not, so either one alone flags healthy boxes
    (profiles/r6_perf_gate.md); a kernel that really got slower misses both."""
    bad_r = check(rows, floors, tol, ratios)
    bad_a = {(k, m) for k, m, _, _ in check(rows, floors, tol)}
    return [b for b in bad_r if not b[1].startswith("ratio_") or (b[0], b[1][len("ratio_"):]) in bad_a
            or b[0] not in floors]


def check(rows, floors: dict, tol: float = 0.03, ratios: typing.Optional[dict] = None):
    """-> list of (key, metric, value, floor) for every floored metric below floor * (1 - tol); higher is better for
    every metric in the floor file (TF/s, PF/s, GB/s and their calibration ratios). A key with ratio floors is
    checked on its ratios (box-independent), one without on its absolute floors."""
    bad = []
    ratios = ratios or {}
    for row in rows:
        key = line_key(row)
        table = ratios.get(key)
        if table:
            table = {"ratio_" + m: f for m, f in table.items()}
        else:
            table = floors.get(key, {})
        for metric, floor in table.items():
            v = row.get(metric)
            if v is None or v < floor * (1.0 - tol):
                bad.append((key, metric, v, floor))
    return bad


def bench_gemm(T: int, reps: int, only=None):
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
        if only is not None and name not in only:
            continue
        A = (torch.randn(M * K, device=dev) * 0.5).to(BF)
        B = (torch.randn(N * K, device=dev) * 0.5).to(BF)
        C = torch.zeros(M * N, device=dev, dtype=torch.float32 if f32 else BF)
        ops = (raw.Operand(A, at, K if at == 0 else M), raw.Operand(B, bt, K if bt == 0 else N), raw.Operand(C, 0, N))
        us = timed(lambda: raw.gemm(*ops, M, N, K), reps)
        fl = 2.0 * M * N * K
        emit(kernel="gemm", shape=name, M=M, N=N, K=K, a_t=at, b_t=bt, out_f32=f32, us_gemm4w=round(us, 1),
             tflops_gemm4w=round(fl / us / 1e6, 1))
        del A, B, C


def bench_mixer(reps: int, only=None):
    """the learned token mixer's GEMMs (K03, ctx32_mixer: 32 x 2048 tokens, 8 heads x 256) on gemm4w: y = tril(W) x
    (tri 1), dx = tril(W)^T dy (tri 2) and the weight gradient dW = dy . x^T over the split (batch, feature)
    contraction index into the lower-triangle tiles (kin = F, tri 3); effective TF/s count only the causal half"""
    B, S, H, Fd = 32, 2048, 8, 256
    dev = torch.device("cuda")
    x = (torch.randn(B * S * H * Fd, device=dev) * 0.5).to(BF)
    w = torch.tril((torch.randn(H, S, S, device=dev) * 0.05)).to(BF).reshape(-1)
    y = torch.empty_like(x)
    gw = torch.zeros(H * S * S, device=dev)
    hf = H * Fd
    fl = B * H * S * S * Fd   # 2 * S * S / 2 per (batch, head, feature)
    for name, a_t, tri in (("mixer y=tril(W)x", 0, 1), ("mixer dx=tril(W)^T dy", 1, 2)):
        if only is not None and name not in only:
            continue

        def run():
            raw.gemm(raw.Operand(w, a_t, S, 0, S * S), raw.Operand(x, 1, hf, S * hf, Fd),
                     raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=tri)
        us = timed(run, reps)
        emit(kernel="gemm", shape=name, us_gemm4w=round(us, 1), tflops_gemm4w=round(fl / us / 1e6, 1))

    def wgrad():
        raw.gemm(raw.Operand(y, 0, hf, 0, Fd), raw.Operand(x, 0, hf, 0, Fd), raw.Operand(gw, 0, S, 0, S * S),
                 S, S, B * Fd, batch=(1, H), beta=1.0, tri=3, kin=Fd, a_sk=S * hf, b_sk=S * hf)
    if only is not None and "mixer dW=dy.x^T (kin, tri 3)" not in only:
        return
    us = timed(wgrad, reps)
    emit(kernel="gemm", shape="mixer dW=dy.x^T (kin, tri 3)", us_gemm4w=round(us, 1),
         tflops_gemm4w=round(fl / us / 1e6, 1))


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
    flash = raw.attn_map_flash_bwd(B, S, H, D, True, False)
    # flash backward: per-batch dS slabs, written whole (no zeroing); map kernels: zeroed per-slice partial sums
    bs = B if flash else raw.attn_map_bsplit(B, S, H)
    pb = torch.zeros(bs, H, S, S, device=dev) if bs > 1 else None
    sc = D ** -0.5
    unit = B * H * S * S / 2 * D * 2
    f = timed(lambda: raw.attn_map_fwd(q, k, v, o, lse, bias, None, B, S, H, D, sc, True), reps)

    def bwd():
        if pb is not None and not flash:
            pb.zero_()
        raw.attn_map_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, bias, None, db, None, B, S, H, D, sc, True, pb)
    b = timed(bwd, reps)
    emit(kernel="attention_map(biased_softmax)", B=B, S=S, H=H, D=D, causal=True, us_fwd=round(f, 1),
         us_bwd=round(b, 1), pflops_fwd=round(2 * unit / f / 1e9, 3), pflops_bwd=round(5 * unit / b / 1e9, 3),
         bias_grad_slices=bs, flash_bwd=flash)


def bench_norm(T: int, reps: int, only=None):
    F = 2048
    dev = torch.device("cuda")
    x = (torch.randn(T * F, device=dev) * 2).to(BF)
    dy, r = ((torch.randn(T * F, device=dev)).to(BF) for _ in range(2))
    sc, sh = torch.ones(F, device=dev), torch.zeros(F, device=dev)
    y, dx = torch.empty_like(x), torch.empty_like(x)
    stats = torch.empty(2 * T, device=dev)
    dsc, dsh = torch.zeros(F, device=dev), torch.zeros(F, device=dev)
    if only is None or "norm_fwd" in only:
        us = timed(lambda: raw.norm_fwd(x, sc, sh, y, stats, T, F, 1), reps)
        emit(kernel="norm_fwd", rows=T, F=F, us=round(us, 1), gbps=round(2 * T * F * 2 / us / 1e3, 1))
    else:   # the backward reads the forward's statistics
        raw.norm_fwd(x, sc, sh, y, stats, T, F, 1)
    for name, R, params in (("norm_bwd+R+params", r, True), ("norm_bwd+R", r, False), ("norm_bwd", None, False)):
        if only is not None and name not in only:
            continue
        args = (dsc, dsh) if params else (None, None)
        us = timed(lambda: raw.norm_bwd(x, dy, sc, stats, dx, args[0], args[1], T, F, 1, F, R=R), reps)
        nbytes = (3 + (1 if R is not None else 0)) * T * F * 2
        emit(kernel=name, rows=T, F=F, us=round(us, 1), gbps=round(nbytes / us / 1e3, 1))


def bench_ew(T: int, reps: int, only=None):
    n = T * 8192
    dev = torch.device("cuda")
    x, z = ((torch.randn(n, device=dev)).to(BF) for _ in range(2))
    y = torch.empty_like(x)
    for name, fn, streams in (("gelu_fwd", lambda: raw.elementwise("act", x, y, act="gelu"), 2),
                              ("gelu_bwd", lambda: raw.elementwise("act_bwd", x, y, z=z, act="gelu"), 3),
                              ("add", lambda: raw.elementwise("add", x, y, z=z), 3)):
        if only is not None and name not in only:
            continue
        us = timed(fn, reps)
        emit(kernel=name, elements=n, us=round(us, 1), gbps=round(streams * n * 2 / us / 1e3, 1))


# The in-suite perf gate (tests/test_gpu_perf_gate.py, `kbench gate`): one row per hot-kernel family, each timed
# between its own two calibrations (short kernels drifted ~3 % against a per-section calibration in round 5)
GATE = (("gemm", "fwd d->4d"), ("gemm", "wgrad logits"), ("mixer", "mixer y=tril(W)x"), ("attn", None),
        ("norm", "norm_bwd"), ("ew", "gelu_bwd"))


def bench_gate(tokens: int, batch: int, reps: int):
    for sec, name in GATE:
        cal0 = calibrate()
        only = None if name is None else {name}
        if sec == "gemm":
            bench_gemm(tokens, reps, only)
        elif sec == "mixer":
            bench_mixer(reps, only)
        elif sec == "attn":
            bench_attn(batch, reps)
        elif sec == "norm":
            bench_norm(tokens, reps, only)
        else:
            bench_ew(tokens, reps, only)
        flush_rows(section_calib(cal0, calibrate()))
        torch.cuda.empty_cache()


def gate_keys():
    return {("attention" if sec == "attn" else (f"gemm {name}" if sec in ("gemm", "mixer") else name))
            for sec, name in GATE}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all", choices=["gemm", "mixer", "attn", "attn_map", "norm", "ew", "all", "gate"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=131072, help="tokens per step (GPT-Neo-1.3B: 64 x 2048)")
    ap.add_argument("--batch", type=int, default=64, help="attention batch at S 2048")
    ap.add_argument("--check", default=None, help="floor file: fail on a regression past --tol")
    ap.add_argument("--tol", type=float, default=0.03)
    ap.add_argument("--write-floors", default=None, help="write the observed ratios as a floor file")
    a = ap.parse_args(argv)
    todo = ["gemm", "mixer", "attn", "attn_map", "norm", "ew"] if a.what == "all" else [a.what]
    if a.what == "gate":
        bench_gate(a.tokens, a.batch, a.reps)
        todo = []
    for w in todo:
        cal0 = calibrate()
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
        flush_rows(section_calib(cal0, calibrate()))
    if a.write_floors:
        out = {"source": "tools/kbench.py --write-floors: observed ratios to the same-process calibration (median of "
                         f"{a.reps} samples)", "floors": {}, "ratios": {}}
        for r in EMITTED:
            k = line_key(r)
            for m in [m for m in r if m.startswith(("tflops", "pflops", "gbps"))]:
                if m.endswith(("hipblaslt", "phase")):
                    continue   # reference implementations are reported, not floored
                out["floors"].setdefault(k, {})[m] = r[m]
                out["ratios"].setdefault(k, {})[m] = r["ratio_" + m]
        with open(a.write_floors, "w") as f:
            json.dump(out, f, indent=1)
    if a.check:
        with open(a.check) as f:
            spec = json.load(f)
        floors, ratios = spec["floors"], spec.get("ratios", {})
        bad = check_either(EMITTED, floors, a.tol, ratios)
        seen = {line_key(r) for r in EMITTED}
        for key, metric, v, floor in bad:
            print(f"REGRESSION {key}: {metric} {v} < floor {floor} - {a.tol:.0%}", flush=True)
        gone = missing(floors, seen, todo) if a.what != "gate" else sorted(gate_keys() - seen)
        for key in gone:
            print(f"MISSING {key}: floored but not emitted by its section", flush=True)
        n = sum(len(m) for k, m in floors.items() if k in seen)
        print(f"kbench check: {n - len(bad)}/{n} floored metrics pass, {len(gone)} floored keys missing", flush=True)
        if bad or gone:
            sys.exit(1)


if __name__ == "__main__":
    main()
