"""Autograd ops for the block-grammar layers off the GPT-Neo hot path, over the kernels of
``csrc/kernels/aux_ops.hip`` (torch oracles of ``ops.raw`` on the CPU):

* ``glu``            K07  a * sigmoid(g)                                   (ref src/model/basic.py:47-57)
* ``product_key``    K14  top-1 per sub-key axis + value-weighted gather   (ref src/model/basic.py:93-115)
* ``moe``            K15  dense soft mixture of experts                    (ref src/model/basic.py:37-44)
* ``sum_axis``       K16  sum over heads                                   (ref src/model/basic.py:77-78)
* ``swap_axes``      K17  transpose_sequence_features via the LDS-tiled transpose kernel (ref basic.py:81-86)
* ``masked_l1``      K24  masked L1 video loss                             (ref src/model/__init__.py:187-199)

Weight gradients follow ``functional``'s convention: accumulated in fp32 straight into ``weight.main_grad``.
"""
from __future__ import annotations

import math
import typing

import torch

from . import raw
from .functional import _acc_grad, _done


def _wgrad_buffer(w: torch.Tensor) -> typing.Tuple[torch.Tensor, bool]:
    if w.dtype == torch.float64:                     # gradient checks: keep fp64 end to end
        return torch.zeros_like(w), False
    return _acc_grad(w)


def _stat_dtype(t: torch.Tensor) -> torch.dtype:
    return torch.float64 if t.dtype == torch.float64 else torch.float32


# ================================================================================================================
class _Glu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, g):
        a, g = a.contiguous(), g.contiguous()
        y = torch.empty_like(a)
        raw.glu(a, g, y)
        ctx.save_for_backward(a, g)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, g = ctx.saved_tensors
        da, dg = torch.empty_like(a), torch.empty_like(g)
        raw.glu(a, g, da, dy=dy.contiguous(), dg=dg)
        return da, dg


def glu(a: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """a * sigmoid(g) in one pass (and both gradients in one pass)"""
    if a.shape != g.shape or a.dtype != g.dtype or (raw.on_gpu(a) and (a.numel() % 8 or a.dtype != torch.bfloat16)):
        return a * torch.sigmoid(g)
    return _Glu.apply(a, g)


# ================================================================================================================
class _ProductKey(torch.autograd.Function):
    @staticmethod
    def forward(ctx, assign, table, R, A, F, H, Fk, P):
        x = assign.contiguous()
        dev = x.device
        sdt = _stat_dtype(x)
        idx = torch.empty(R, dtype=torch.int32, device=dev)
        val = torch.empty(R, dtype=sdt, device=dev)
        stats = torch.empty(R * A * 2, dtype=sdt, device=dev)
        aidx = torch.empty(R * A, dtype=torch.int32, device=dev)
        raw.pkm_top1(x, idx, val, stats, aidx, R, A, F)
        out = torch.empty(R * Fk, dtype=table.dtype, device=dev)
        raw.pkm_gather(idx, val, table, out, R, H, Fk, P)
        ctx.save_for_backward(x, table, idx, val, stats, aidx)
        ctx.cfg = (R, A, F, H, Fk, P)
        ctx.shape = assign.shape
        return out

    @staticmethod
    def backward(ctx, dy):
        x, table, idx, val, stats, aidx = ctx.saved_tensors
        R, A, F, H, Fk, P = ctx.cfg
        gt, is_main = _wgrad_buffer(table)
        dval = torch.empty(R, dtype=val.dtype, device=x.device)
        raw.pkm_gather_bwd(idx, val, table, dy.contiguous(), gt, dval, R, H, Fk, P)
        _done(table)
        dx = torch.empty_like(x)
        raw.pkm_top1_bwd(x, val, dval, stats, aidx, dx, R, A, F)
        return dx.view(ctx.shape), (None if is_main else gt.to(table.dtype)), None, None, None, None, None, None


def product_key(assign: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    """assign [..., H, A, F] (normalised sub-key logits), table [P = F^A, H, Fk] -> [..., H, Fk]:
    out[.., h] = table[sum_a i_a F^a, h] * prod_a softmax_a(x)[i_a], i_a = argmax_f x[.., h, a, f]"""
    *lead, H, A, F = assign.shape
    P, Ht, Fk = table.shape
    if Ht != H or P != F ** A:
        raise ValueError(f"product-key table {list(table.shape)} does not match assignment {list(assign.shape)}")
    R = int(math.prod(lead)) * H
    out = _ProductKey.apply(assign, table, R, A, F, H, Fk, P)
    return out.view(*lead, H, Fk)


def product_key_ok(assign: torch.Tensor, table: torch.Tensor) -> bool:
    if not raw.on_gpu(assign):
        return True
    return (assign.dtype == torch.bfloat16 and table.dtype == torch.bfloat16 and table.shape[-1] % 8 == 0
            and assign.shape[-1] ** assign.shape[-2] < 2 ** 31)


# ================================================================================================================
class _MoE(torch.autograd.Function):
    """y[t][n] = sum_e softmax(lg[t])[e] (x[t] · W[:, n, e]): ONE plain GEMM against the expert-minor weight viewed
    as [K][N*E] (no weight copies), then the softmax + expert contraction kernel; backward: the contraction kernel's
    adjoint (dU = dy ⊗ p, d logits through the softmax Jacobian) and two plain GEMMs for dx and dW"""

    @staticmethod
    def forward(ctx, x, lg, w, T, K, N, E):
        xc, lgc = x.contiguous(), lg.contiguous()
        dev = xc.device
        u = torch.empty(T * N * E, dtype=xc.dtype, device=dev)
        raw.gemm(raw.Operand(xc, 0, K), raw.Operand(w, 1, N * E), raw.Operand(u, 0, N * E), T, N * E, K)
        p = torch.empty(T * E, dtype=_stat_dtype(xc), device=dev)
        y = torch.empty(T * N, dtype=xc.dtype, device=dev)
        raw.moe_fwd(u, lgc, p, y, T, N, E)
        ctx.save_for_backward(xc, w, u, p)
        ctx.cfg = (T, K, N, E, x.shape, lg.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w, u, p = ctx.saved_tensors
        T, K, N, E, xs, ls = ctx.cfg
        du = torch.empty_like(u)
        dlg = torch.empty(T * E, dtype=xc.dtype, device=xc.device)
        raw.moe_bwd(dy.contiguous(), u, p, du, dlg, T, N, E)
        dx = torch.empty(T * K, dtype=xc.dtype, device=xc.device)
        raw.gemm(raw.Operand(du, 0, N * E), raw.Operand(w, 0, N * E), raw.Operand(dx, 0, K), T, K, N * E)
        gw, is_main = _wgrad_buffer(w)
        raw.gemm(raw.Operand(xc, 1, K), raw.Operand(du, 1, N * E), raw.Operand(gw, 0, N * E), K, N * E, T, beta=1.0)
        _done(w)
        return dx.view(xs), dlg.view(ls), (None if is_main else gw.to(w.dtype)), None, None, None, None


def moe_ok(x: torch.Tensor, E: int, K: int) -> bool:
    if not raw.on_gpu(x):
        return True
    return x.dtype == torch.bfloat16 and raw.moe_ok(E) and K % 8 == 0


def moe(x: torch.Tensor, lg: torch.Tensor, w: torch.Tensor, T: int, K: int, N: int, E: int) -> torch.Tensor:
    """x [T, K], gate logits lg [T, E], w [K, N, E] -> [T * N]"""
    return _MoE.apply(x, lg, w, T, K, N, E)


# ================================================================================================================
class _SumAxis(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis):
        xc = x.contiguous()
        shape = list(xc.shape)
        outer, H, inner = int(math.prod(shape[:axis])), shape[axis], int(math.prod(shape[axis + 1:]))
        y = torch.empty(shape[:axis] + shape[axis + 1:], dtype=xc.dtype, device=xc.device)
        raw.sum_axis(xc, y, outer, H, inner)
        ctx.cfg = (axis, shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        axis, shape = ctx.cfg
        return dy.unsqueeze(axis).expand(shape), None


def sum_axis(x: torch.Tensor, axis: int) -> torch.Tensor:
    inner = int(math.prod(x.shape[axis + 1:]))
    if raw.on_gpu(x) and (x.dtype != torch.bfloat16 or inner % 8):
        return x.sum(axis)
    return _SumAxis.apply(x, axis)


# ================================================================================================================
def _swap(x: torch.Tensor, a: int, b: int) -> torch.Tensor:
    """y = x.transpose(a, b) materialised, for the last axis b and x.shape[a] == x.shape[b] (y has x's shape)"""
    shape = list(x.shape)
    outer = int(math.prod(shape[:a]))
    S, F = shape[a], shape[b]
    mid = int(math.prod(shape[a + 1:b]))
    y = torch.empty_like(x)
    xf, yf = x.reshape(-1), y.reshape(-1)
    blk = S * mid * F
    if mid == 1:          # [outer][S][F] -> [outer][F][S]
        raw.transpose(xf, yf, S, F, F, S, batch=outer, sx=blk, sy=blk)
        return y
    for o in range(outer):   # x[o][s][m][f] -> y[o][f][m][s]: per (o), batch over m
        raw.transpose(xf[o * blk:], yf[o * blk:], S, F, mid * F, mid * S, batch=mid, sx=F, sy=S)
    return y


class _SwapAxes(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, b):
        ctx.cfg = (a, b)
        return _swap(x.contiguous(), a, b)

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.cfg
        return _swap(dy.contiguous(), a, b), None, None


def swap_axes(x: torch.Tensor, a: int, b: int) -> torch.Tensor:
    """x.transpose(a, b).contiguous() for equal-sized axes (transpose_sequence_features); the HIP transpose kernel on
    the GPU when b is the last axis and the sizes are multiples of 8"""
    a, b = min(a, b), max(a, b)
    shape = list(x.shape)
    mid = int(math.prod(shape[a + 1:b]))
    if (not raw.on_gpu(x) or x.dtype != torch.bfloat16 or b != x.dim() - 1 or shape[a] != shape[b]
            or shape[a] % 8 or (mid * shape[b]) % 8):
        return x.transpose(a, b).contiguous()
    return _SwapAxes.apply(x, a, b)


# ================================================================================================================
class _MaskedL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fo, g, mask, inner):
        foc, gc = fo.contiguous(), g.contiguous()
        loss = torch.zeros(1, dtype=_stat_dtype(foc), device=foc.device)
        raw.l1(foc, gc, mask, inner, loss=loss)
        ctx.save_for_backward(foc, gc, mask)
        ctx.inner = inner
        return loss[0]

    @staticmethod
    def backward(ctx, dl):
        foc, gc, mask = ctx.saved_tensors
        dfo = torch.empty_like(foc)
        gptr = dl.reshape(1).to(torch.float32 if raw.on_gpu(foc) else dl.dtype).contiguous()
        raw.l1(foc, gc, mask, ctx.inner, dfo=dfo, gptr=gptr)
        return dfo, None, None, None


def masked_l1(fo: torch.Tensor, g: torch.Tensor, mask: typing.Optional[torch.Tensor]) -> torch.Tensor:
    """sum |(fo - g) * mask| with ``mask`` over fo's leading dims (None: no mask); gradient sign(.) * mask"""
    n = fo.numel()
    if mask is not None:
        mask = mask.to(torch.float64 if fo.dtype == torch.float64 else torch.float32).contiguous()
        if list(fo.shape[:mask.dim()]) != list(mask.shape):
            raise ValueError(f"mask {list(mask.shape)} must cover the leading dims of {list(fo.shape)}")
    inner = n // (mask.numel() if mask is not None else 1)
    if raw.on_gpu(fo) and (fo.dtype != torch.bfloat16 or g.dtype != torch.bfloat16):
        out = fo.float() - g.float()
        if mask is not None:
            out = out * mask.view(list(mask.shape) + [1] * (out.dim() - mask.dim()))
        return (out * torch.sign(out.detach())).sum()
    return _MaskedL1.apply(fo, g, mask, inner)
