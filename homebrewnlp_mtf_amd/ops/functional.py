"""Autograd ops of the model, written once against ``ops.raw`` (HIP on GPU, torch oracle on CPU).

Weight gradients never go through autograd: every op adds its fp32 weight gradient straight into the flat gradient
buffer (``weight.main_grad``, see ``models/variables.py``) with a beta=1 GEMM epilogue (beta=0 for the first
contribution of a step) and returns ``None`` -- this
is the MI355X-native replacement of the reference's per-variable gradient einsums (src/optimizer/__init__.py:128-174)
and lets the DP all-reduce start on contiguous buckets while backward is still running.

TP collectives are issued where the reference's ``heads`` layout implies them:
  * linear contracting ``heads`` (row-parallel, X01/X03/X04): all-reduce the output in forward;
  * linear creating ``heads`` from replicated input (column-parallel, X02): all-reduce dX in backward;
  * non-group norm (X05): all-reduce row statistics in forward and backward.
"""
from __future__ import annotations

import functools
import math
import typing

import torch

from . import raw
from ..config import Dim
from ..parallel import state as pstate

DimList = typing.List[Dim]


def _empty(shape, like: torch.Tensor, dtype=None):
    return torch.empty(shape, dtype=dtype or like.dtype, device=like.device)


GRAD_HOOK: typing.Optional[typing.Callable[[torch.Tensor], None]] = None   # set by parallel.grad_sync


def _acc_grad(w: torch.Tensor) -> typing.Tuple[torch.Tensor, bool]:
    """(fp32 buffer to accumulate the weight gradient into, whether it is the flat main_grad)"""
    mg = getattr(w, "main_grad", None)
    if mg is not None:
        fresh = getattr(getattr(w, "store", None), "fresh", None)
        if fresh is not None:
            fresh.discard(w.var_name)
        return mg, True
    return torch.zeros(w.shape, dtype=torch.float32, device=w.device), False


def _acc_grad_beta(w: torch.Tensor) -> typing.Tuple[torch.Tensor, bool, float]:
    """like ``_acc_grad`` plus the GEMM beta: 0 (overwrite) for the first contribution of the step to a flat-buffer
    gradient, 1 (accumulate) after that: an fp32 weight-gradient GEMM without the C read-back ran up to 13 % faster
    (round 2, tools/lab/bench_wgrad.py, profiles/r2_wgrad_layouts.txt)."""
    mg = getattr(w, "main_grad", None)
    if mg is None:
        return torch.zeros(w.shape, dtype=torch.float32, device=w.device), False, 0.0
    fresh = getattr(getattr(w, "store", None), "fresh", None)
    first = fresh is not None and w.var_name in fresh
    if fresh is not None:
        fresh.discard(w.var_name)
    return mg, True, 0.0 if first else 1.0


def _param32(t: typing.Optional[torch.Tensor]) -> typing.Optional[torch.Tensor]:
    """small parameters (norm scale/shift, rezero gate) are read from the fp32 master copy; fp64 (gradient-check)
    computations use the tensor itself"""
    if t is None or t.dtype == torch.float64:
        return t
    m = getattr(t, "master", t)
    return m if m.dtype == torch.float32 else m.float()


def _done(w: torch.Tensor):
    """a weight-gradient contribution has been accumulated (DP bucket bookkeeping)"""
    if GRAD_HOOK is not None:
        GRAD_HOOK(w)


# ================================================================================================================
# named linear  y[P, S, N] = sum_C x[P, S, C] * w[S, C, N]   (S = shared/batch dims, e.g. heads of `group`)
class LinearPlan:
    def __init__(self, xdims: DimList, wdims: DimList, odims: DimList, head_name: str = "heads"):
        xs, ws, os_ = list(xdims), list(wdims), list(odims)
        self.S = [d for d in ws if d in xs and d in os_]
        self.C = [d for d in ws if d in xs and d not in os_]
        self.Nn = [d for d in ws if d not in xs]
        self.P = [d for d in xs if d not in ws]
        if ws != self.S + self.C + self.Nn:
            raise NotImplementedError(f"weight dims {ws} not in [shared, contracted, new] order")
        canon_x = self.P + self.S + self.C
        canon_o = self.P + self.S + self.Nn
        if sorted(os_) != sorted(canon_o):
            raise ValueError(f"output dims {os_} inconsistent with x {xs} / w {ws}")
        self.x_perm = None if xs == canon_x else [xs.index(d) for d in canon_x]
        self.o_perm = None if os_ == canon_o else [canon_o.index(d) for d in os_]
        self.canon_o_shape = [d.size for d in canon_o]
        self.out_shape = [d.size for d in os_]
        prod = lambda ds: int(math.prod(d.size for d in ds))  # noqa: E731
        self.M, self.H, self.K, self.N = prod(self.P), prod(self.S), prod(self.C), prod(self.Nn)
        # TP roles (heads axis split over ranks)
        names_c = [d.name for d in self.C]
        names_n = [d.name for d in self.Nn]
        self.row_parallel = head_name in names_c          # contracts heads -> partial sums
        self.col_parallel = head_name in names_n          # creates heads from replicated input


@functools.lru_cache(maxsize=4096)
def linear_plan(xdims: tuple, wdims: tuple, odims: tuple) -> LinearPlan:
    return LinearPlan(list(xdims), list(wdims), list(odims))


# Operand layouts on the GPU. The MFMA kernels' K-contiguous (ds_read_b128) path beats the transposed-read path and
# lets gemm4w keep its row-layout (TLAY) epilogue, so the forward reads a cached [N][K] copy of the weight; gemm4w
# reads the token-strided layouts of the weight gradient at full rate, so x and dy are not transposed
# (`OBST_TRANSPOSED_OPERANDS=0` turns the weight copies off for A/B measurements).
_KCONTIG = __import__("os").environ.get("OBST_TRANSPOSED_OPERANDS", "1") != "0"
# Refreshing every copy costs one transpose pass over the bf16 weights per step (~1 ms); decode-step products
# (M = 32 tokens, skinny.hip) need the K-contiguous copy too.
# OBST_ATTN_FUSED_RESIDUAL=0: the attention block's residual add as a separate elementwise pass (A/B)
_ATTN_RES = __import__("os").environ.get("OBST_ATTN_FUSED_RESIDUAL", "1") == "1"


def _wT(w, plan: LinearPlan, act=None, has_r: bool = False):
    store = getattr(w, "store", None)
    if not _KCONTIG or store is None or not raw.on_gpu(w) or w.dtype != torch.bfloat16:
        return None
    if plan.K % 8 or plan.N % 8:
        return None
    return store.transposed(w.var_name, plan.H, plan.K, plan.N)


def _fwd_gemm(x2, w, y2, plan: LinearPlan, act=None, R=None, Zout=None, alpha: float = 1.0):
    M, H, K, N = plan.M, plan.H, plan.K, plan.N
    wt = _wT(w, plan, act, R is not None)
    bop = raw.Operand(wt, 0, K, K * N) if wt is not None else raw.Operand(w, 1, N, K * N)
    raw.gemm(raw.Operand(x2, 0, H * K, K), bop, raw.Operand(y2, 0, H * N, N),
             M, N, K, batch=(H, 1), act=act, R=R, Zout=Zout, alpha=alpha)


# Row-parallel forward under TP (the weight contracts the sharded heads: every rank holds a partial sum of the whole
# output): the product runs in OBST_TP_CHUNKS token blocks and each block's all-reduce starts on RCCL's stream as soon
# as its GEMM is done, so the next block's GEMM overlaps it -- only the last block's all-reduce stays exposed. Blocks
# stay >= 4096 tokens (a whole number of 256-row tiles, ~full-rate GEMMs). Opt-in (default 1 block): the persistent
# GEMM loses about the run time of any kernel that holds CUs beside it (profiles/r4_cu_contention.md) and splitting
# adds tile tails, so the overlap is unproven until a TP > 1 RCCL measurement shows a gain.
_TP_CHUNKS = max(int(__import__("os").environ.get("OBST_TP_CHUNKS", "1")), 1)
_TP_MIN_ROWS = int(__import__("os").environ.get("OBST_TP_MIN_ROWS", "4096"))   # (tests: tiny blocks)


def tp_chunks(M: int) -> typing.List[typing.Tuple[int, int]]:
    """[m0, m1) token blocks of the chunked row-parallel forward"""
    c = _TP_CHUNKS
    while c > 1 and (M // c < _TP_MIN_ROWS):
        c //= 2
    step = -(-M // c)
    step = -(-step // 256) * 256 if _TP_MIN_ROWS >= 256 else step
    return [(m0, min(m0 + step, M)) for m0 in range(0, M, step)]


def _fwd_gemm_reduced(x2, w, y2, plan: LinearPlan):
    """y2 = x2 . w summed over the TP group (row-parallel plan): token blocks, each block's all-reduce overlapping
    the next block's GEMM (identity reduction when tp == 1)"""
    if pstate.tp_size() == 1 or x2.device.type == "meta":
        _fwd_gemm(x2, w, y2, plan)
        pstate.tp_all_reduce(y2)
        return
    M, H, K, N = plan.M, plan.H, plan.K, plan.N
    xf, yf = x2.reshape(M, H * K), y2.view(M, H * N)
    wt = _wT(w, plan, None, False)
    bop = raw.Operand(wt, 0, K, K * N) if wt is not None else raw.Operand(w, 1, N, K * N)
    pending = []
    for m0, m1 in tp_chunks(M):
        yc = yf[m0:m1]
        raw.gemm(raw.Operand(xf[m0:m1], 0, H * K, K), bop, raw.Operand(yc, 0, H * N, N), m1 - m0, N, K, batch=(H, 1))
        pending.append(pstate.tp_all_reduce_async(yc))
    for h in pending:
        h.wait()


def tokens_transposed(x2, rows: int, cols: int) -> typing.Optional[torch.Tensor]:
    """[rows][cols] bf16 -> [cols][rows] (None where the plain transposed-read GEMM is used instead)"""
    if not _KCONTIG or not raw.on_gpu(x2) or x2.dtype != torch.bfloat16 or rows % 8 or cols % 8:
        return None
    if raw.on_gpu(x2):   # gemm4w reads the token-strided layouts at full rate
        return None
    out = torch.empty(cols * rows, dtype=x2.dtype, device=x2.device)
    raw.transpose(x2, out, rows, cols, cols, rows)
    return out


def _dgrad_gemm(dy2, w, dx2, plan: LinearPlan, act=None, Zin=None, R=None):
    M, H, K, N = plan.M, plan.H, plan.K, plan.N
    raw.gemm(raw.Operand(dy2, 0, H * N, N), raw.Operand(w, 0, N, K * N), raw.Operand(dx2, 0, H * K, K),
             M, K, N, batch=(H, 1), act=act, act_bwd=Zin is not None, Zin=Zin, R=R)


def _wgrad_gemm(x2, dy2, gw, plan: LinearPlan, xT=None, dyT=None, beta: float = 1.0):
    """gw[H][K][N] (+)= x[M][H][K]ᵀ · dy[M][H][N] (beta 0: overwrite, 1: accumulate); with token-contiguous
    transposes (xT [H*K][M], dyT [H*N][M]) the operands are K-contiguous"""
    M, H, K, N = plan.M, plan.H, plan.K, plan.N
    if xT is None:
        xT = tokens_transposed(x2, M, H * K)
    if xT is not None and dyT is None:
        dyT = tokens_transposed(dy2, M, H * N)
    if xT is not None and dyT is not None:
        raw.gemm(raw.Operand(xT, 0, M, K * M), raw.Operand(dyT, 0, M, N * M), raw.Operand(gw, 0, N, K * N),
                 K, N, M, batch=(H, 1), beta=beta)
        return
    if xT is not None:      # shared token-contiguous x (round 2: NT ran ~25 % faster than TT at T = 32k)
        raw.gemm(raw.Operand(xT, 0, M, K * M), raw.Operand(dy2, 1, H * N, N), raw.Operand(gw, 0, N, K * N),
                 K, N, M, batch=(H, 1), beta=beta)
        return
    raw.gemm(raw.Operand(x2, 1, H * K, K), raw.Operand(dy2, 1, H * N, N), raw.Operand(gw, 0, N, K * N),
             K, N, M, batch=(H, 1), beta=beta)


class StreamSink:
    """The RevNet stream update of a block fused into the block's last GEMM (ref src/model/revnet.py:20-49): forward
    y2 = x1 + F(x2) (alpha 1), backward reconstruction x1 = y2 - F(x2) (alpha -1), out of that GEMM's epilogue instead
    of a separate pass over the stream. fp32 stream: ``out32`` = r + alpha * F in fp32 plus its bf16 copy, which the op
    returns -- a value autograd never reads: the RevNet stack back-propagates dL/dF through that op explicitly. bf16
    stream (``revnet_stream_dtype`` "calculation"): r + alpha * F in bf16 is the op's output itself. Either way
    ``out`` holds the updated stream once an op has consumed the sink."""

    def __init__(self, r: torch.Tensor, alpha: float):
        self.r, self.alpha = r, float(alpha)
        self.out32: typing.Optional[torch.Tensor] = None
        self.out: typing.Optional[torch.Tensor] = None

    def usable(self, y_shape, device) -> bool:
        """a fresh fp32 / bf16 stream buffer of the op's output shape on the GPU, nothing consumed yet"""
        return (self.out is None and raw.on_gpu(self.r) and self.r.dtype in (torch.float32, torch.bfloat16)
                and self.r.is_contiguous() and self.r.numel() == math.prod(y_shape) and self.r.device == device)

    def run(self, y_shape, device, gemm) -> torch.Tensor:
        """gemm(y, R, Zout, alpha): the fused product; returns the op's bf16 output"""
        y16 = torch.empty(y_shape, dtype=torch.bfloat16, device=device)
        if self.r.dtype == torch.bfloat16:
            gemm(y16, self.r, None, self.alpha)
            self.out = y16
            return y16
        y32 = torch.empty(y_shape, dtype=torch.float32, device=device)
        gemm(y32, self.r, y16, self.alpha)
        self.out32 = self.out = y32
        return y16


class ReluGrad:
    """A relu-activated product whose output feeds a norm: the norm backward multiplies its dx by [x > 0] (x = the
    relu output it normalised, so that is relu'(z)) and marks ``applied``; the product's backward (which runs after)
    then takes that gradient as dz and skips its own activation-backward pass."""
    __slots__ = ("applied",)

    def __init__(self):
        self.applied = False


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, plan: LinearPlan, act, sink: typing.Optional[StreamSink] = None,
                relu_grad: typing.Optional[ReluGrad] = None):
        xc = x.permute(plan.x_perm).contiguous() if plan.x_perm is not None else x.contiguous()
        z = _empty(plan.canon_o_shape, xc) if act else None
        if plan.row_parallel and pstate.tp_size() > 1:
            if act:
                raise NotImplementedError("activation fused into a heads-contracting linear under TP")
            y = _empty(plan.canon_o_shape, xc)
            _fwd_gemm_reduced(xc, w, y, plan)
        elif (sink is not None and act is None and plan.o_perm is None
              and sink.usable(plan.canon_o_shape, xc.device)):
            y = sink.run(plan.canon_o_shape, xc.device,
                         lambda yo, R, Z, a: _fwd_gemm(xc, w, yo, plan, R=R, Zout=Z, alpha=a))
        else:
            y = _empty(plan.canon_o_shape, xc)
            _fwd_gemm(xc, w, y, plan, act=act, Zout=z)
        ctx.save_for_backward(xc, w, z)
        ctx.plan, ctx.act = plan, act
        ctx.relu_grad = relu_grad if act == "relu" else None
        if plan.o_perm is not None:
            y = y.permute(plan.o_perm)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w, z = ctx.saved_tensors
        plan, act = ctx.plan, ctx.act
        if plan.o_perm is not None:
            inv = [plan.o_perm.index(i) for i in range(len(plan.o_perm))]
            dy = dy.permute(inv)
        dy = dy.contiguous()
        if act and not (ctx.relu_grad is not None and ctx.relu_grad.applied):
            dz = torch.empty_like(dy)
            raw.elementwise("act_bwd", z, dz, z=dy, act=act)
            dy = dz
        ctx.relu_grad = None
        dx = None
        pending = pstate._DONE
        if ctx.needs_input_grad[0]:
            dx = _empty(xc.shape, xc)
            _dgrad_gemm(dy, w, dx, plan)
            if plan.col_parallel and pstate.tp_size() > 1:
                pending = pstate.tp_all_reduce_async(dx)   # overlaps the weight-gradient GEMM below
            if plan.x_perm is not None:
                inv = [plan.x_perm.index(i) for i in range(len(plan.x_perm))]
                dx = dx.permute(inv)
        gw, is_main, beta = _acc_grad_beta(w)
        _wgrad_gemm(xc, dy, gw, plan, beta=beta)
        _done(w)
        pending.wait()
        return dx, (None if is_main else gw.to(w.dtype)), None, None, None, None


def linear(x: torch.Tensor, w: torch.Tensor, xdims: DimList, wdims: DimList, odims: DimList,
           act: typing.Optional[str] = None, sink: typing.Optional[StreamSink] = None,
           relu_grad: typing.Optional[ReluGrad] = None) -> torch.Tensor:
    plan = linear_plan(tuple(xdims), tuple(wdims), tuple(odims))
    return _Linear.apply(x, w, plan, act, sink, relu_grad)


class _TPReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return pstate.tp_all_reduce(x.contiguous().clone())

    @staticmethod
    def backward(ctx, dy):
        return dy


class _TPCopy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, dy):
        return pstate.tp_all_reduce(dy.contiguous().clone())


def tp_reduce(x):
    """all-reduce over the TP group in forward, identity in backward (row-parallel output)"""
    return _TPReduce.apply(x) if pstate.tp_size() > 1 else x


def tp_copy(x):
    """identity in forward, all-reduce of the gradient in backward (column-parallel input)"""
    return _TPCopy.apply(x) if pstate.tp_size() > 1 else x


# ================================================================================================================
# fused feed-forward: y = act(x W1) W2 (+ residual)   -- K01 x4 with fused epilogues, no separate elementwise pass
class _FFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, w2, p1: LinearPlan, p2: LinearPlan, act, residual, carrier=None):
        xc = x.contiguous()
        tp = pstate.tp_size() > 1
        z = _empty(p1.canon_o_shape, xc)
        a = _empty(p1.canon_o_shape, xc) if act else z
        if tp and p1.row_parallel:
            # W1 contracts the sharded heads: the pre-activation is a partial sum -- reduce it, then activate
            _fwd_gemm_reduced(xc, w1, z, p1)
            if act:
                raw.elementwise("act", z, a, act=act)
        else:
            _fwd_gemm(xc, w1, a, p1, act=act, Zout=z if act else None)
        y = _empty(p2.canon_o_shape, xc)
        if tp and p2.row_parallel:   # partial output: reduce before the residual joins
            _fwd_gemm_reduced(a, w2, y, p2)
            if residual is not None:
                raw.elementwise("add", y, y, z=residual.contiguous())
        else:
            _fwd_gemm(a, w2, y, p2, R=residual.contiguous() if residual is not None else None)
        ctx.save_for_backward(xc, w1, w2, z, a if act else None)
        ctx.p1, ctx.p2, ctx.act, ctx.has_res = p1, p2, act, residual is not None
        ctx.carrier = carrier
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, w1, w2, z, a = ctx.saved_tensors
        p1, p2, act = ctx.p1, ctx.p2, ctx.act
        a = z if a is None else a
        dy = dy.contiguous()
        # dZ = (dY W2^T) * act'(Z) in ONE gemm epilogue
        tp = pstate.tp_size() > 1
        dz = _empty(p1.canon_o_shape, dy)
        # act'(z) is the same on every TP rank (z is replicated), so the fused act-backward epilogue commutes with
        # the all-reduce of the partial dz (W2 contracting the sharded heads)
        _dgrad_gemm(dy, w2, dz, p2, act=act, Zin=z if act else None)
        # TP: each data-gradient all-reduce runs on RCCL's stream under the weight-gradient GEMM that follows it
        pending = pstate.tp_all_reduce_async(dz) if tp and p2.col_parallel else pstate._DONE
        g2, m2, b2 = _acc_grad_beta(w2)
        _wgrad_gemm(a, dy, g2, p2, beta=b2)
        _done(w2)
        pending.wait()
        dx = _empty(xc.shape, xc)
        _dgrad_gemm(dz, w1, dx, p1)
        pending = pstate.tp_all_reduce_async(dx) if tp and p1.col_parallel else pstate._DONE
        g1, m1, b1 = _acc_grad_beta(w1)
        _wgrad_gemm(xc, dz, g1, p1, beta=b1)
        _done(w1)
        pending.wait()
        dres = dy if ctx.has_res else None
        if dres is not None and ctx.carrier is not None:   # handed to the block's opening norm (ResidualGrad)
            ctx.carrier.grad, dres = dres, None
        return (dx, None if m1 else g1.to(w1.dtype), None if m2 else g2.to(w2.dtype), None, None, None, dres, None)


class _FFNItp(torch.autograd.Function):
    """Feed-forward with the intermediate axis split over the TP group (``tp_layout: "intermediate"``):
    the input's heads are gathered (all-gather [T, d/tp] -> [T, d]), both GEMMs run on this rank's slice of the
    intermediate, and the partial output is reduce-scattered back to this rank's heads; backward mirrors it
    (all-gather dy, reduce-scatter dx). Wire bytes per layer and direction: 2 T d (x (tp-1)/tp) against 2 T I for
    the reference layout's all-reduce of the replicated [T, I] intermediate -- 4x fewer at I = 4d."""

    @staticmethod
    def forward(ctx, x, w1, w2, p1: LinearPlan, p2: LinearPlan, act, residual, carrier=None):
        T = p1.M
        dl = x.numel() // T
        xf = pstate.tp_gather_rows(x.contiguous().view(T, dl), T, dl)
        z = _empty(p1.canon_o_shape, xf)
        a = _empty(p1.canon_o_shape, xf) if act else z
        _fwd_gemm(xf, w1, a, p1, act=act, Zout=z if act else None)
        yf = _empty([T, p2.N], xf)
        _fwd_gemm(a, w2, yf, p2)
        y = pstate.tp_reduce_scatter_rows(yf, T, dl).view(x.shape)
        if residual is not None:
            raw.elementwise("add", y, y, z=residual.contiguous())
        ctx.save_for_backward(xf, w1, w2, z, a if act else None)
        ctx.p1, ctx.p2, ctx.act, ctx.has_res, ctx.carrier = p1, p2, act, residual is not None, carrier
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        xf, w1, w2, z, a = ctx.saved_tensors
        p1, p2, act = ctx.p1, ctx.p2, ctx.act
        a = z if a is None else a
        T = p1.M
        dl = dy.numel() // T
        dyf = pstate.tp_gather_rows(dy.contiguous().view(T, dl), T, dl)
        dz = _empty(p1.canon_o_shape, dyf)
        _dgrad_gemm(dyf, w2, dz, p2, act=act, Zin=z if act else None)
        g2, m2, b2 = _acc_grad_beta(w2)
        _wgrad_gemm(a, dyf, g2, p2, beta=b2)
        _done(w2)
        dxf = _empty([T, p1.H * p1.K], dyf)
        _dgrad_gemm(dz, w1, dxf, p1)
        dx = pstate.tp_reduce_scatter_rows(dxf, T, dl).view(ctx.xshape)
        g1, m1, b1 = _acc_grad_beta(w1)
        _wgrad_gemm(xf, dz, g1, p1, beta=b1)
        _done(w1)
        dres = dy if ctx.has_res else None
        if dres is not None and ctx.carrier is not None:
            ctx.carrier.grad, dres = dres, None
        return (dx, None if m1 else g1.to(w1.dtype), None if m2 else g2.to(w2.dtype), None, None, None, dres, None)


def ffn_itp(x, w1, w2, xg_dims, w1dims, mdims, w2dims, og_dims, act, residual=None, carrier=None):
    """x: this rank's heads; xg_dims / og_dims: the same dims with the global heads (what the GEMMs see)"""
    p1 = linear_plan(tuple(xg_dims), tuple(w1dims), tuple(mdims))
    p2 = linear_plan(tuple(mdims), tuple(w2dims), tuple(og_dims))
    if p1.x_perm is not None or p1.o_perm is not None or p2.x_perm is not None or p2.o_perm is not None:
        raise NotImplementedError("intermediate-split FFN needs canonical layouts")
    return _FFNItp.apply(x, w1, w2, p1, p2, act, residual, carrier)


def ffn(x, w1, w2, xdims, w1dims, mdims, w2dims, odims, act, residual=None, carrier=None):
    p1 = linear_plan(tuple(xdims), tuple(w1dims), tuple(mdims))
    p2 = linear_plan(tuple(mdims), tuple(w2dims), tuple(odims))
    if p1.x_perm is not None or p1.o_perm is not None or p2.x_perm is not None or p2.o_perm is not None:
        raise NotImplementedError("fused FFN needs canonical layouts")
    return _FFN.apply(x, w1, w2, p1, p2, act, residual, carrier)


# ================================================================================================================
# fused dot-product attention block (reference spatial.py:42-81 with 'dot_product', 'context'/'embedded' keys):
#   base = act(x W_in);  k, q, v = base W_k, base W_q, base W_v;  out = softmax(q k^T * scale, causal) v (+ residual)
class _DotAttention(torch.autograd.Function):
    """k, q and v live interleaved in ONE token-major buffer kqv[T][3N] (row = k | q | v of a token; the attention
    kernels take the 3N row stride), so with the three weights adjacent in the flat buffer (the registration order)
      forward : kqv = base · [W_k W_q W_v]           -- one GEMM, N = 3N, on the stacked K-contiguous weight copies
      dgrad   : dbase = dkqv · [W_k W_q W_v]ᵀ         -- one GEMM, K = 3N, no residual-input chaining
      wgrad   : dW_j = baseᵀ · dkqv[:, jN:(j+1)N]     -- three GEMMs on column slices (3N row stride)
    (GPT-Neo-1.3B: the three dgrads took 4.96 ms per layer as one plain + two residual-chained products)."""

    @staticmethod
    def forward(ctx, x, w_in, w_k, w_q, w_v, p_in: LinearPlan, p_out: LinearPlan, act, scale, causal, residual,
                geo, carrier=None):
        B, S, H, D = geo
        xc = x.contiguous()
        base = _empty(p_in.canon_o_shape, xc)
        z = _empty(p_in.canon_o_shape, xc) if act else None
        if p_in.row_parallel and pstate.tp_size() > 1:
            # partial sums over the sharded heads: reduce the pre-activation, then activate
            pre = z if act else base
            _fwd_gemm(xc, w_in, pre, p_in)
            pstate.tp_all_reduce(pre)
            if act:
                raw.elementwise("act", z, base, act=act)
        else:
            _fwd_gemm(xc, w_in, base, p_in, act=act, Zout=z)
        T, K, N = p_out.M, p_out.K, p_out.N
        kqv = _empty([T, 3 * N], xc)
        _kqv_fwd(base, (w_k, w_q, w_v), kqv, p_out)
        k, q, v = kqv[:, 0:N], kqv[:, N:2 * N], kqv[:, 2 * N:]
        o = _empty(p_out.canon_o_shape, xc)
        lse = torch.empty(B * H * S, dtype=torch.float32, device=xc.device)
        if residual is not None and _ATTN_RES:   # the residual add rides in the attention epilogue (o kept: backward)
            out = torch.empty_like(o)
            raw.attn_fwd(q, k, v, o, lse, B, S, H, D, 3 * N, scale, causal, ld_o=H * D,
                         residual=residual.contiguous(), out=out)
        else:
            raw.attn_fwd(q, k, v, o, lse, B, S, H, D, 3 * N, scale, causal, ld_o=H * D)
            out = o
            if residual is not None:
                out = torch.empty_like(o)
                raw.elementwise("add", o, out, z=residual.contiguous())
        ctx.save_for_backward(xc, w_in, w_k, w_q, w_v, z, base, kqv, o, lse)
        ctx.cfg = (p_in, p_out, act, scale, causal, geo, residual is not None)
        ctx.carrier = carrier
        return out

    @staticmethod
    def backward(ctx, dout):
        xc, w_in, w_k, w_q, w_v, z, base, kqv, o, lse = ctx.saved_tensors
        p_in, p_out, act, scale, causal, (B, S, H, D), has_res = ctx.cfg
        dout = dout.contiguous()
        T, K, N = p_out.M, p_out.K, p_out.N
        k, q, v = kqv[:, 0:N], kqv[:, N:2 * N], kqv[:, 2 * N:]
        dkqv = torch.empty_like(kqv)
        delta = torch.empty(B * H * S, dtype=torch.float32, device=xc.device)
        raw.attn_bwd(q, k, v, o, dout, lse, delta, dkqv[:, N:2 * N], dkqv[:, 0:N], dkqv[:, 2 * N:], B, S, H, D,
                     3 * N, scale, causal, ld_o=H * D)
        ws = (w_k, w_q, w_v)
        dbase = _empty(p_in.canon_o_shape, xc)
        _kqv_dgrad(dkqv, ws, dbase, p_out, act, z)
        # TP: act'(z) is replicated, so the activation-backward fused into the dgrad commutes with the sum; the
        # all-reduce of the partial dbase runs on RCCL's stream under the three k/q/v weight-gradient GEMMs
        pending = (pstate.tp_all_reduce_async(dbase) if p_out.col_parallel and pstate.tp_size() > 1
                   else pstate._DONE)
        baseT = None   # (gemm4w reads the token-strided base at full rate: no transpose)
        outs = []
        for j in range(3):
            g, m, bj = _acc_grad_beta(ws[j])
            dyj = dkqv[:, j * N:(j + 1) * N]
            a_op = raw.Operand(baseT, 0, T, K * T) if baseT is not None else raw.Operand(base, 1, K, K * T)
            raw.gemm(a_op, raw.Operand(dyj, 1, 3 * N), raw.Operand(g, 0, N, K * N), K, N, T, beta=bj)
            _done(ws[j])
            outs.append(None if m else g.to(ws[j].dtype))
        pending.wait()
        dx = _empty(xc.shape, xc)
        _dgrad_gemm(dbase, w_in, dx, p_in)
        g, m, bi = _acc_grad_beta(w_in)
        _wgrad_gemm(xc, dbase, g, p_in, beta=bi)
        _done(w_in)
        dres = dout if has_res else None
        if dres is not None and ctx.carrier is not None:   # handed to the block's opening norm (ResidualGrad)
            ctx.carrier.grad, dres = dres, None
        return (dx, None if m else g.to(w_in.dtype), outs[0], outs[1], outs[2], None, None, None, None, None,
                dres, None, None)


def _kqv_cat(w, K: int, N: int):
    """[K][3N] row interleave of the stacked [3][K][N] q / k / v weights (one strided-copy kernel)"""
    cat = torch.empty((K, 3 * N), dtype=w.dtype, device=w.device)
    raw.copy2d(w, cat, K, N, N, 3 * N, batch=3, sx=K * N, sy=N)
    return cat


def _stacked(ws) -> bool:
    """the three weights are equal-sized blocks adjacent in the flat buffer, in order (registration order)"""
    w0 = ws[0]
    n = w0.numel()
    es = w0.element_size()
    return (all(w.is_contiguous() and w.numel() == n for w in ws) and ws[1].data_ptr() - w0.data_ptr() == n * es
            and ws[2].data_ptr() - ws[1].data_ptr() == n * es)


def _kqv_fwd(base, ws, kqv, p: LinearPlan):
    """kqv[T][3N] = base · [W_k W_q W_v]"""
    M, H, K, N = p.M, p.H, p.K, p.N
    if H != 1:
        raise NotImplementedError("interleaved k|q|v projection needs plain [K][N] weights")
    wt = _wT(ws[0], p) if _stacked(ws) else None
    if wt is not None:
        for j in (1, 2):
            _wT(ws[j], p)           # refresh the neighbours' transposed copies (adjacent to wt: a [3N][K] stack)
        raw.gemm(raw.Operand(base, 0, K), raw.Operand(wt, 0, K), raw.Operand(kqv, 0, 3 * N), M, 3 * N, K)
        return
    if _stacked(ws):   # one batched launch: C block j at column offset j*N of the 3N-wide rows
        raw.gemm(raw.Operand(base, 0, K, 0), raw.Operand(ws[0], 1, N, K * N), raw.Operand(kqv, 0, 3 * N, N),
                 M, N, K, batch=(3, 1))
        return
    for j in range(3):
        raw.gemm(raw.Operand(base, 0, K), raw.Operand(ws[j], 1, N), raw.Operand(kqv[:, j * N:], 0, 3 * N), M, N, K)


def _kqv_dgrad(dkqv, ws, dbase, p: LinearPlan, act, z):
    """dbase = act'(z) * (dkqv · [W_k W_q W_v]ᵀ): on the GPU ONE GEMM over K = 3N whose B operand is the weights
    concatenated along N ([K][3N], derived once per step); elsewhere three products chained through the residual
    input"""
    M, K, N = p.M, p.K, p.N
    w0 = ws[0]
    store = getattr(w0, "store", None)
    if raw.on_gpu(dkqv) and store is not None and _stacked(ws):
        cat = store.derived(w0.var_name, f"kqv_cat@{w0.data_ptr()}", lambda: _kqv_cat(w0.detach(), K, N))
        raw.gemm(raw.Operand(dkqv, 0, 3 * N), raw.Operand(cat, 0, 3 * N), raw.Operand(dbase, 0, K), M, K, 3 * N,
                 act=act, act_bwd=act is not None, Zin=z if act else None)
        return
    for j in range(3):
        last = j == 2
        raw.gemm(raw.Operand(dkqv[:, j * N:], 0, 3 * N), raw.Operand(ws[j], 0, N), raw.Operand(dbase, 0, K),
                 M, K, N, act=act if last else None, act_bwd=last and act is not None,
                 Zin=z if (last and act) else None, R=dbase if j > 0 else None)


def dot_attention(x, w_in, w_k, w_q, w_v, xdims, w_in_dims, base_dims, w_out_dims, act, scale, causal, geo,
                  residual=None, carrier=None):
    p_in = linear_plan(tuple(xdims), tuple(w_in_dims), tuple(base_dims))
    p_out = linear_plan(tuple(base_dims), tuple(w_out_dims), tuple(xdims))
    if p_out.H != 1:   # decided before any GEMM or collective runs (the caller falls back to the generic path)
        raise NotImplementedError("interleaved k|q|v projection needs plain [K][N] weights")
    return _DotAttention.apply(x, w_in, w_k, w_q, w_v, p_in, p_out, act, scale, causal, residual, geo, carrier)


# ================================================================================================================
# K03: learned token mixer (reference `attention-biased_attention_map-...-input_as_value`, spatial.py:19-23,72-81)
#   y[b,s,h,f] = sum_{s'} (W[h,s,s'] * M[s,s']) x[b,s',h,f],   M = lower triangle incl. the diagonal when causal
# One strided two-level-batched GEMM per pass (batch = batch x heads); the causal triangle is skipped tile-wise
# (tri flags of the GEMM), so forward and dgrad run ~half the dense FLOPs and dW only fills the lower triangle.
class _TokenMixer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, causal: bool, sink: typing.Optional[StreamSink] = None):
        B, S, H, Fd = x.shape
        xc = x.contiguous()
        store = getattr(w, "store", None)
        if causal and store is not None and w.device.type == "cuda":
            # the masked weight of a depth-shared mixer is built once per step (ParamStore.derived)
            wm = store.derived(w.var_name, f"tril@{w.data_ptr()}", lambda: raw.tril(w.detach()))
        else:
            wm = torch.tril(w) if causal else w.contiguous()
        hf = H * Fd

        def product(y, R=None, Zout=None, alpha=1.0):
            raw.gemm(raw.Operand(wm, 0, S, 0, S * S), raw.Operand(xc, 1, hf, S * hf, Fd),
                     raw.Operand(y, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=1 if causal else 0,
                     R=R, Zout=Zout, alpha=alpha)
        if sink is not None and sink.usable(xc.shape, xc.device):
            y = sink.run(xc.shape, xc.device, lambda yo, R, Z, a: product(yo, R=R, Zout=Z, alpha=a))
        else:
            y = torch.empty_like(xc)
            product(y)
        ctx.save_for_backward(xc, wm, w)
        ctx.causal = causal
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wm, w = ctx.saved_tensors
        B, S, H, Fd = xc.shape
        hf = H * Fd
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(xc)
            raw.gemm(raw.Operand(wm, 1, S, 0, S * S), raw.Operand(dy, 1, hf, S * hf, Fd),
                     raw.Operand(dx, 0, hf, S * hf, Fd), S, Fd, S, batch=(B, H), tri=2 if ctx.causal else 0)
        g, m = _acc_grad(w)
        # dW[h] = dy_h · x_hᵀ over (batch, features), both read in place from [B, S, H, F]: the contraction index
        # (b, f) is split (kin = F contiguous features, outer stride S*H*F), so no [H][S][B*F] copies are made
        kk = B * Fd
        if raw.on_gpu(dy) and B == 1:
            # one sequence: the contraction runs over the F contiguous features of each row -- plain row-strided
            # operands, no split index
            raw.gemm(raw.Operand(dy, 0, hf, 0, Fd), raw.Operand(xc, 0, hf, 0, Fd), raw.Operand(g, 0, S, 0, S * S),
                     S, S, Fd, batch=(1, H), beta=1.0, tri=3 if ctx.causal else 0)
        elif raw.on_gpu(dy) and Fd % 64 == 0 and S % 8 == 0 and (B % 2 == 0 or not ctx.causal):
            # (the causal product runs as >= 2 split-K slabs that start on whole (b, f) blocks: B even)
            raw.gemm(raw.Operand(dy, 0, hf, 0, Fd), raw.Operand(xc, 0, hf, 0, Fd), raw.Operand(g, 0, S, 0, S * S),
                     S, S, kk, batch=(1, H), beta=1.0, tri=3 if ctx.causal else 0, kin=Fd, a_sk=S * hf, b_sk=S * hf)
        else:
            dyp = dy.permute(2, 1, 0, 3).reshape(H, S, B * Fd).contiguous()
            xp = xc.permute(2, 1, 0, 3).reshape(H, S, B * Fd).contiguous()
            raw.gemm(raw.Operand(dyp, 0, kk, 0, S * kk), raw.Operand(xp, 0, kk, 0, S * kk),
                     raw.Operand(g, 0, S, 0, S * S), S, S, kk, batch=(1, H), beta=1.0, tri=3 if ctx.causal else 0)
        _done(w)
        return dx, (None if m else g.to(w.dtype)), None, None


def token_mixer(x, w, causal: bool, sink: typing.Optional[StreamSink] = None):
    """x [B, S, H, F], w [H, S, S] (query, key); sink: the RevNet stream update fused into the product"""
    return _TokenMixer.apply(x, w, causal, sink)


@torch.no_grad()
def token_mixer_step(x_new, xc, wm, pos):
    """one decode step of the token mixer: x_new [B, 1, H, F] joins the cached inputs xc [B, S, H, F] at pos [B];
    returns y [B, 1, H, F] with y[b, 0, h] = wm[h, pos[b], :] · xc[b, :, h] (wm masked: entries past pos are 0)"""
    B, _, H, Fd = x_new.shape
    S = xc.shape[1]
    rows = torch.arange(B, device=xc.device)
    xc[rows, pos] = x_new[:, 0].to(xc.dtype)
    wr = wm.index_select(1, pos).permute(1, 0, 2).contiguous()        # [B, H, S]: the query rows
    y = torch.empty(B, 1, H, Fd, dtype=x_new.dtype, device=x_new.device)
    hf = H * Fd
    raw.gemm(raw.Operand(wr, 0, S, H * S, S), raw.Operand(xc, 1, hf, S * hf, Fd), raw.Operand(y, 0, hf, hf, Fd),
             1, Fd, S, batch=(B, H))
    return y


@torch.no_grad()
def cumsum_step(x_new, csum, pos, mean: bool):
    """one decode step of cumsum / cummean: csum [B, S, ...] fp32 running sums (updated at pos [B])"""
    B = x_new.shape[0]
    rows = torch.arange(B, device=csum.device)
    prev = csum[rows, (pos - 1).clamp(min=0)]
    prev = torch.where((pos > 0).view([B] + [1] * (prev.dim() - 1)), prev, torch.zeros_like(prev))
    cur = prev + x_new[:, 0].float()
    csum[rows, pos] = cur
    if mean:
        cur = cur / (pos + 1).to(cur.dtype).view([B] + [1] * (cur.dim() - 1))
    return cur.to(x_new.dtype).unsqueeze(1)


# ================================================================================================================
# general attention core on already-projected q, k, v [B, S, H, D] (used by the composable attention path)
class _AttnCore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal):
        B, S, H, D = q.shape
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o = torch.empty_like(q)
        lse = torch.empty(B * H * S, dtype=torch.float32, device=q.device)
        raw.attn_fwd(q, k, v, o, lse, B, S, H, D, H * D, scale, causal)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (scale, causal)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale, causal = ctx.cfg
        B, S, H, D = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        delta = torch.empty(B * H * S, dtype=torch.float32, device=q.device)
        raw.attn_bwd(q, k, v, o, do.contiguous(), lse, delta, dq, dk, dv, B, S, H, D, H * D, scale, causal)
        return dq, dk, dv, None, None


def attention_core(q, k, v, scale: float, causal: bool):
    return _AttnCore.apply(q, k, v, scale, causal)


_MAP_WS = {}


def _map_workspace(device, numel: int) -> torch.Tensor:
    """per-device fp32 scratch of the attention-map backward (reused across calls). Grown only outside stream
    capture: a buffer first allocated under capture belongs to the graph's private pool, so it is handed out for
    that capture alone and never cached for eager calls (the trainer's eager warm-up step sizes the cache)."""
    ws = _MAP_WS.get(device)
    if ws is None or ws.numel() < numel:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return torch.empty(numel, dtype=torch.float32, device=device)
        ws = _MAP_WS[device] = torch.empty(numel, dtype=torch.float32, device=device)
    return ws[:numel]


def release_workspaces() -> None:
    """drop the cached per-device scratch buffers (attention-map backward); the next call re-allocates"""
    _MAP_WS.clear()


class _AttnMap(torch.autograd.Function):
    """flash attention with per-head [H, S, S] maps (raw.attn_map_*): bias added to the scaled logits, cmap
    multiplied into the softmax probabilities; either may be None. No [B, H, S, S] tensor is formed on the GPU."""

    @staticmethod
    def forward(ctx, q, k, v, bias, cmap, scale, causal):
        B, S, H, D = q.shape
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        md = torch.float64 if q.dtype == torch.float64 else torch.float32   # fp64: the CPU gradient checks
        b32 = bias.to(md).contiguous() if bias is not None else None
        c32 = cmap.to(md).contiguous() if cmap is not None else None
        o = torch.empty_like(q)
        lse = torch.empty(B * H * S, dtype=md, device=q.device)
        raw.attn_map_fwd(q, k, v, o, lse, b32, c32, B, S, H, D, scale, causal)
        ctx.save_for_backward(q, k, v, o, lse, b32, c32)
        ctx.cfg = (scale, causal, bias.dtype if bias is not None else None, cmap.dtype if cmap is not None else None)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, b32, c32 = ctx.saved_tensors
        scale, causal, bdt, cdt = ctx.cfg
        B, S, H, D = q.shape
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        md = lse.dtype
        delta = torch.empty(B * H * S, dtype=md, device=q.device)
        need_b = b32 is not None and ctx.needs_input_grad[3]
        need_c = c32 is not None and ctx.needs_input_grad[4]
        db = torch.empty(H, S, S, dtype=md, device=q.device) if need_b else None
        dc = torch.empty(H, S, S, dtype=md, device=q.device) if need_c else None
        pb = pc = None
        if raw.on_gpu(q) and raw.attn_map_flash_bwd(B, S, H, D, b32 is not None, c32 is not None):
            # flash backward with the map hook: dS per batch, written whole (no zeroing), folded by the kernel
            pb = _map_workspace(q.device, B * H * S * S).view(B, H, S, S)
        elif raw.on_gpu(q) and (need_b or need_c):
            bs = raw.attn_map_bsplit(B, S, H)
            if bs > 1:
                # the per-batch-slice partial map gradients live in one cached workspace (reused by every layer's
                # backward, stream-ordered; ~1 GiB per map at S 2048 H 16 bsplit 4 was allocated per call)
                n = bs * H * S * S
                ws = _map_workspace(q.device, n * (int(need_b) + int(need_c)))
                ws.zero_()
                parts = iter(ws.split(n))
                pb = next(parts).view(bs, H, S, S) if need_b else None
                pc = next(parts).view(bs, H, S, S) if need_c else None
        raw.attn_map_bwd(q, k, v, o, do.contiguous(), lse, delta, dq, dk, dv, b32, c32, db, dc, B, S, H, D, scale,
                         causal, pb, pc)
        return (dq, dk, dv, db.to(bdt) if db is not None else None, dc.to(cdt) if dc is not None else None,
                None, None)


class _Axial(torch.autograd.Function):
    """K12 axial positional embedding: [n_0, .., n_{k-1}, F] = broadcast product of k factor tables [n_m, F]"""

    @staticmethod
    def forward(ctx, F_, *tables):
        ts = [t.contiguous() for t in tables]
        n = [t.numel() // F_ for t in ts]
        out = torch.empty(math.prod(n) * F_, dtype=ts[0].dtype, device=ts[0].device)
        raw.axial_fwd(ts, out, F_)
        ctx.save_for_backward(*ts)
        ctx.F = F_
        return out.view(n + [F_])

    @staticmethod
    def backward(ctx, g):
        ts = ctx.saved_tensors
        md = torch.float64 if g.dtype == torch.float64 else torch.float32
        grads = [torch.empty(t.numel(), dtype=md, device=g.device) for t in ts]
        raw.axial_bwd(ts, g.contiguous(), grads, ctx.F)
        return (None,) + tuple(gr.view(t.shape).to(t.dtype) for gr, t in zip(grads, ts))


def axial_embed(tables, F: int):
    return _Axial.apply(F, *tables)


def attention_map(q, k, v, bias, cmap, scale: float, causal: bool):
    return _AttnMap.apply(q, k, v, bias, cmap, scale, causal)


# ================================================================================================================
# norm
class ResidualGrad:
    """Carries a pre-norm block's residual-input gradient from the fused op that consumed the residual (FFN /
    attention epilogue) to the norm that opens the block on the same input tensor: the norm backward adds it into dx
    inside its kernel, so autograd does not sum the two gradients of the block input with a separate elementwise
    pass. The consumer's backward always runs first (the norm's output feeds it)."""
    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None


class GradSink:
    """The RevNet stream gradient of a block input (ref src/model/revnet.py:51-120): the norm opening the block adds
    the stream gradient g into its dx inside the backward kernel -- fp32 stream: the sum in fp32 (``out32``) plus the
    bf16 copy it returns as dx; bf16 stream: dx itself -- replacing the separate dx2 = g1 + dF/dx2 pass. ``out32`` holds
    the fp32 sum; ``ptr`` is the address of the bf16 dx the norm returned: the stack checks that the
    input's .grad is exactly it (no other gradient was summed in). ``fused``: the norm consumed the sink (bf16
    stream: the sum is the input's .grad itself)."""

    def __init__(self, g: torch.Tensor):
        self.g = g
        self.out32: typing.Optional[torch.Tensor] = None
        self.out: typing.Optional[torch.Tensor] = None
        self.fused = False
        self.ptr = 0

    def usable(self, x: torch.Tensor) -> bool:
        return (not self.fused and raw.on_gpu(self.g) and self.g.dtype in (torch.float32, torch.bfloat16)
                and self.g.is_contiguous() and self.g.numel() == x.numel() and self.g.device == x.device)


class _Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, shift, F, groups, tp_stats, carrier=None, grad_sink=None, act=None, relu_grad=None):
        xc = x.contiguous()
        rows = xc.numel() // F
        y = torch.empty_like(xc)
        stats = torch.empty(2 * rows, dtype=torch.float32, device=xc.device)
        sm32 = _param32(scale)
        sh32 = _param32(shift)
        ext = None
        Ffull = F
        if tp_stats and pstate.tp_size() > 1:
            part = torch.empty(2 * rows, dtype=torch.float32, device=xc.device)
            raw.norm_partial(xc, part, rows, F)
            pstate.tp_all_reduce(part)
            Ffull = F * pstate.tp_size()
            p = part.view(rows, 2)
            mean = p[:, 0] / Ffull
            var = (p[:, 1] / Ffull - mean * mean).clamp_min(0)
            ext = torch.stack([mean, torch.rsqrt(var + raw.EPS)], -1).reshape(-1).contiguous()
        if act is not None and ext is not None:
            raise NotImplementedError("activation fused into a TP-statistics norm")
        raw.norm_fwd(xc, sm32, sh32, y, stats, rows, F, groups, ext_stats=ext, act=act)
        ctx.save_for_backward(xc, scale, shift, stats)
        ctx.act, ctx.sh32 = act, sh32
        ctx.relu_grad = relu_grad if ext is None else None
        ctx.cfg = (F, groups, rows, Ffull, tp_stats)
        ctx.sm32 = sm32
        ctx.carrier = carrier
        ctx.grad_sink = grad_sink
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, scale, shift, stats = ctx.saved_tensors
        F, groups, rows, Ffull, tp_stats = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty_like(xc)
        gsc, msc = _acc_grad(scale) if scale is not None else (None, True)
        gsh, msh = _acc_grad(shift) if shift is not None else (None, True)
        ext = None
        if tp_stats and pstate.tp_size() > 1:
            part = torch.empty(2 * rows, dtype=torch.float32, device=xc.device)
            raw.norm_bwd(xc, dy, ctx.sm32, stats, None, None, None, rows, F, groups, Ffull, partial=part)
            pstate.tp_all_reduce(part)
            ext = part
        R = None
        if ctx.carrier is not None and ctx.carrier.grad is not None:
            R = ctx.carrier.grad.contiguous()
            ctx.carrier.grad = None
        sink = ctx.grad_sink
        rg = ctx.relu_grad
        ctx.relu_grad = None
        if ctx.act is not None or (rg is not None and ext is None):
            # the fused activation (dy through act'(z)) and / or the producer's relu (dx * [x > 0]) in the kernel
            raw.norm_bwd(xc, dy, ctx.sm32, stats, dx, gsc, gsh, rows, F, groups, Ffull, R=R, shift=ctx.sh32,
                         act=ctx.act, in_relu=rg is not None)
            if rg is not None:
                rg.applied = True
        elif sink is not None and R is None and ext is None and sink.usable(xc):
            if sink.g.dtype == torch.bfloat16:   # bf16 stream: dx = norm gradient + stream gradient
                raw.norm_bwd(xc, dy, ctx.sm32, stats, dx, gsc, gsh, rows, F, groups, Ffull, R=sink.g)
                # (no reference to dx kept here: autograd's AccumulateGrad steals a gradient only when nothing else
                # holds it, else it copies it into .grad -- 0.76 ms per block at ctx32_mixer's batch 256)
                sink.fused = True
            else:
                dx32 = torch.empty(xc.shape, dtype=torch.float32, device=xc.device)
                raw.norm_bwd(xc, dy, ctx.sm32, stats, dx, gsc, gsh, rows, F, groups, Ffull, R32=sink.g, dx32=dx32)
                sink.out32 = sink.out = dx32
            sink.fused = True
            sink.ptr = dx.data_ptr()
        else:
            raw.norm_bwd(xc, dy, ctx.sm32, stats, dx, gsc, gsh, rows, F, groups, Ffull, ext_dsum=ext, R=R)
        ctx.grad_sink = None
        for t in (scale, shift):
            if t is not None:
                _done(t)
        return (dx, None if msc else gsc.view(scale.shape).to(scale.dtype),
                None if msh else gsh.view(shift.shape).to(shift.dtype), None, None, None, None, None, None, None)


def norm(x, scale, shift, F: int, groups: int, tp_stats: bool = False, carrier: typing.Optional[ResidualGrad] = None,
         grad_sink: typing.Optional[GradSink] = None, act: typing.Optional[str] = None,
         relu_grad: typing.Optional[ReluGrad] = None):
    """act: the activation layer that follows the norm, applied in the norm kernel (and its derivative in the norm's
    backward, from z recomputed out of the row statistics) instead of two elementwise passes"""
    return _Norm.apply(x, scale, shift, F, groups, tp_stats, carrier, grad_sink, act, relu_grad)


# ================================================================================================================
# elementwise autograd ops
class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        raw.elementwise("act", xc, y, act=act)
        ctx.save_for_backward(xc)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        (xc,) = ctx.saved_tensors
        dx = torch.empty_like(xc)
        raw.elementwise("act_bwd", xc, dx, z=dy.contiguous(), act=ctx.act)
        return dx, None


def activation(x, act: typing.Optional[str]):
    if act in (None, "none", "identity"):
        return x
    return _Act.apply(x, act)


class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        raw.elementwise("add", a, y, z=b)
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


def add(a, b):
    if a.shape != b.shape:
        return a + b
    return _Add.apply(a, b)


class _Rezero(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        sm = _param32(g).reshape(-1)
        raw.elementwise("mul_scalar", xc, y, sptr=sm)
        ctx.save_for_backward(xc, g)
        ctx.sm = sm
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, g = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        raw.elementwise("mul_scalar", dy, dx, sptr=ctx.sm)
        gg, m = _acc_grad(g)
        raw.dot(xc, dy, gg.reshape(-1))
        _done(g)
        return dx, None if m else gg.to(g.dtype)


def rezero(x, g):
    return _Rezero.apply(x, g)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, keep, seed):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        raw.elementwise("dropout", xc, y, keep=keep, seed=seed)
        ctx.cfg = (keep, seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        keep, seed = ctx.cfg
        dx = torch.empty_like(dy.contiguous())
        raw.elementwise("dropout", dy.contiguous(), dx, keep=keep, seed=seed)
        return dx, None, None


def dropout(x, keep: float, seed: int, train: bool = True):
    if not train or keep >= 1.0:
        return x
    return _Dropout.apply(x, keep, seed)


class _Cumsum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis, mean):
        xc = x.contiguous()
        shape = xc.shape
        outer = int(math.prod(shape[:axis]))
        S = shape[axis]
        inner = int(math.prod(shape[axis + 1:]))
        y = torch.empty_like(xc)
        raw.cumsum(xc, y, outer, S, inner, reverse=False, mean=mean, grad=False)
        ctx.cfg = (outer, S, inner, mean)
        return y

    @staticmethod
    def backward(ctx, dy):
        outer, S, inner, mean = ctx.cfg
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        raw.cumsum(dy, dx, outer, S, inner, reverse=True, mean=mean, grad=True)
        return dx, None, None


def cumsum(x, axis: int, mean: bool = False):
    return _Cumsum.apply(x, axis, mean)


# ================================================================================================================
# embedding gather (K08) / scatter-add (K09)
class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, table, V, F):
        idx32 = idx.to(torch.int32).contiguous()
        T = idx32.numel()
        out = torch.empty(list(idx.shape) + [F], dtype=table.dtype, device=table.device)
        raw.gather(idx32, table, out, T, F, V)
        ctx.save_for_backward(idx32, table)
        ctx.cfg = (T, F, V)
        return out

    @staticmethod
    def backward(ctx, dy):
        idx32, table = ctx.saved_tensors
        T, F, V = ctx.cfg
        g, m = _acc_grad(table)
        raw.scatter_add(idx32, dy.contiguous(), g, T, F, V)
        _done(table)
        return None, None if m else g.to(table.dtype), None, None


def gather(idx, table, V: int, F: int):
    return _Gather.apply(idx, table, V, F)


# ================================================================================================================
# fused output projection + softmax cross-entropy + z-loss + accuracy (K01 + K10)
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, tgt, V, z_loss, n_total):
        rows = tgt.numel()
        Vp = logits.shape[-1]
        lc = logits.contiguous()
        t32 = tgt.to(torch.int32).contiguous()
        sdt = torch.float64 if lc.dtype == torch.float64 else torch.float32
        lse = torch.empty(rows, dtype=sdt, device=lc.device)
        loss = torch.empty(rows, dtype=sdt, device=lc.device)
        hit = torch.empty(rows, dtype=sdt, device=lc.device)
        raw.xent_fwd(lc, t32, lse, loss, hit, rows, V, Vp, z_loss)
        ctx.save_for_backward(lc, t32, lse)
        ctx.cfg = (rows, V, Vp, z_loss, n_total)
        ctx.mark_non_differentiable(hit)
        return loss.sum() / n_total, hit.sum() / n_total

    @staticmethod
    def backward(ctx, dloss, dacc):
        lc, t32, lse = ctx.saved_tensors
        rows, V, Vp, z_loss, n_total = ctx.cfg
        g = lc  # in-place: the logits buffer is dead after this point
        gptr = dloss.reshape(1).to(lse.dtype).contiguous()
        raw.xent_bwd(lc, t32, lse, g, gptr, 1.0 / n_total, rows, V, Vp, z_loss)
        return g, None, None, None, None


def softmax_xent(logits, tgt, V: int, z_loss: float, n_total: int):
    """(mean loss incl. z-loss, accuracy). `logits` may be vocab-padded (columns >= V ignored)."""
    return _SoftmaxXent.apply(logits, tgt, V, z_loss, n_total)
