#!/usr/bin/env python3
"""Per-GEMM census of one training step: every ``raw.gemm`` launch of the bench model is timed with HIP events and
grouped by signature (M, N, K, operand layouts, output dtype, beta, residual, batch), so the weak GEMM shapes of the
real step show up with their achieved TFLOP/s.

    python tools/gemm_census.py [--config configs/gpt_neo_1.3b.json] [--batch-per-gpu 64]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from homebrewnlp_mtf_amd.config import load_config  # noqa: E402
from homebrewnlp_mtf_amd.ops import raw  # noqa: E402
from homebrewnlp_mtf_amd.parallel import state as pstate  # noqa: E402
from homebrewnlp_mtf_amd.run.trainer import Trainer  # noqa: E402

_orig = raw.gemm
_stack = []
_records = []
_on = [False]


def _wrapped(a, b, c, M, N, K, batch=(1, 1), alpha=1.0, beta=0.0, act=None, act_bwd=False, R=None, Zout=None,
             Zin=None, tri=0, **kw):
    if not _on[0]:
        return _orig(a, b, c, M, N, K, batch, alpha, beta, act, act_bwd, R, Zout, Zin, tri, **kw)
    frame = {"nested": False}
    if _stack:
        _stack[-1]["nested"] = True
    _stack.append(frame)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = _orig(a, b, c, M, N, K, batch, alpha, beta, act, act_bwd, R, Zout, Zin, tri, **kw)
    e1.record()
    _stack.pop()
    if not frame["nested"]:
        sig = (M, N, K, a.trans, b.trans, a.ld, b.ld, str(c.t.dtype)[6:], beta != 0.0, R is not None,
               batch[0] * batch[1], act or "", int(act_bwd), tri, int(kw.get("kin", 0) or 0))
        _records.append((sig, e0, e1))
    return out


_orig_t = raw.transpose
_trecords = []


def _wrapped_t(x, y, rows, cols, ldx, ldy, batch=1, sx=0, sy=0):
    if not _on[0]:
        return _orig_t(x, y, rows, cols, ldx, ldy, batch, sx, sy)
    import traceback
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = _orig_t(x, y, rows, cols, ldx, ldy, batch, sx, sy)
    e1.record()
    caller = traceback.extract_stack(limit=3)[0]
    _trecords.append(((rows, cols, batch, f"{os.path.basename(caller.filename)}:{caller.lineno}"), e0, e1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/gpt_neo_1.3b.json")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    args = ap.parse_args()
    raw.gemm = _wrapped
    raw.transpose = _wrapped_t
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh = pstate.Mesh(dp=1, tp=1, rank=0).build_groups()
    params = load_config(args.config, {"train_batch_size": args.batch_per_gpu, "mesh": {"dp": 1, "tp": 1}})
    torch.manual_seed(0)
    tr = Trainer(params, dev, mesh)
    S = params.sequence_length
    toks = torch.randint(0, params.vocab_size, (args.batch_per_gpu, S + 1, 1), device=dev)
    batch = {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    _on[0] = True
    tr.step(batch)
    torch.cuda.synchronize()
    _on[0] = False
    agg = collections.OrderedDict()
    for sig, e0, e1 in _records:
        ms = e0.elapsed_time(e1)
        n, t = agg.get(sig, (0, 0.0))
        agg[sig] = (n + 1, t + ms)
    total = sum(t for _, t in agg.values())
    print(f"{len(_records)} GEMM launches, {total:.1f} ms (event-bracketed, includes launch gaps)")
    print("| M | N | K | a_t | b_t | lda | ldb | out | beta | R | batch | act | bwd | tri | calls | ms | us/call | TF/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for sig, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        M, N, K = sig[0], sig[1], sig[2]
        fl = 2.0 * M * N * K * sig[10] * n
        print("| " + " | ".join(str(s) for s in sig) + f" | {n} | {t:.2f} | {1000 * t / n:.0f} | {fl / t / 1e9:.0f} |")
    tagg = collections.OrderedDict()
    for sig, e0, e1 in _trecords:
        n, t = tagg.get(sig, (0, 0.0))
        tagg[sig] = (n + 1, t + e0.elapsed_time(e1))
    print(f"\n{len(_trecords)} transposes, {sum(t for _, t in tagg.values()):.1f} ms")
    print("| rows | cols | batch | caller | calls | ms | us/call | GB/s |")
    print("|---|---|---|---|---|---|---|---|")
    for sig, (n, t) in sorted(tagg.items(), key=lambda kv: -kv[1][1]):
        gb = 4.0 * sig[0] * sig[1] * sig[2] * n / 1e9
        print("| " + " | ".join(str(s) for s in sig) + f" | {n} | {t:.2f} | {1000 * t / n:.0f} | {gb / t * 1e3:.0f} |")


if __name__ == "__main__":
    main()
