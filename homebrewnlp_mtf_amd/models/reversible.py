"""Memory-reduction strategies of the body: ``revnet``, ``momentum``, ``checkpoint`` and ``none``
(ref src/model/__init__.py:94-130, src/model/revnet.py:14-120, src/model/momentumnet.py:14-125).

RevNet (reversible residual): state (x1, x2) -> (x2, x1 + F(x2)); the body returns x1 + x2. The whole depth stack
is ONE autograd node: forward keeps no activations, backward walks the blocks in reverse, reconstructs
x1 = y2 - F(x2), re-runs F(x2) with grad enabled and back-propagates through it (weight gradients land in the flat
fp32 buffer via the ops' fused wgrad epilogues). Activation memory is O(1) in depth, as in the reference.

MomentumNet: v' = a v + (1-a) F(x); x' = x + v'; inverse v = (v' - (1-a) F(x)) / a, x = x' - v'.

Each block is re-entered in backward under the exact scope it ran in (``Scope.restore``) so it fetches the same
variables by name (incl. ``shared`` cross-depth reuse).
"""
from __future__ import annotations

import typing

import torch

from ..ops import functional as F
from ..ops import raw
from ..utils import debug
from .context import Act, Builder
from .frontend import block_body, block_scope_name


class Block:
    def __init__(self, builder: Builder, config, depth: int, config_idx: int, stack: typing.List[str], dims):
        self.builder, self.config, self.depth, self.config_idx = builder, config, depth, config_idx
        self.stack = stack + [block_scope_name(depth, config_idx)]
        self.dims = dims

    def __call__(self, x: torch.Tensor, sink=None, gsink=None) -> torch.Tensor:
        b = self.builder
        b.depth_idx, b.config_idx = self.depth, self.config_idx
        with b.scope.restore(self.stack), debug.range_(self.stack[-1]):
            return block_body(b, self.config, Act(x, self.dims), stream_sink=sink, grad_sink=gsink).t


# OBST_REV_FUSE=0: the RevNet stream updates as separate mix_f32 passes (A/B)
_REV_FUSE = __import__("os").environ.get("OBST_REV_FUSE", "1") != "0"


def _sink(r32: torch.Tensor, alpha: float):
    return F.StreamSink(r32, alpha) if _REV_FUSE and raw.on_gpu(r32) else None


def _stream_dtype(dt: torch.dtype, calc: bool = False) -> torch.dtype:
    """fp32 streams (fp64 for the fp64 oracle); ``calc`` (revnet_stream_dtype "calculation"): the compute dtype"""
    if calc:
        return dt
    return torch.float64 if dt == torch.float64 else torch.float32


def _add(a, b, beta: float = 1.0):
    """a + beta * b in a's dtype (one elementwise pass)"""
    if raw.on_gpu(a) and a.dtype == torch.bfloat16:
        return _axpby(a, b, 1.0, beta)
    return a + beta * b


def _sum_to(a, b, dt):
    """(a + b) in dtype dt: one fused fp32 + fp32 -> bf16 pass on the GPU (raw.add_to_bf16), bf16 + bf16 through
    the HIP axpby"""
    if dt == torch.bfloat16 and raw.on_gpu(a):
        if a.dtype == torch.float32 and b.dtype == torch.float32:
            return raw.add_to_bf16(a, b)
        if a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16:
            return _add(a, b)
    return (a + b).to(dt)


def _to_stream(x, sd):
    """the body input as a stream: bf16 -> fp32 through the HIP cast kernel on the GPU"""
    if sd == torch.float32 and x.dtype == torch.bfloat16 and raw.on_gpu(x):
        return raw.to_f32(x)
    return x.to(sd)


def _axpby(x, z, alpha, beta):
    y = torch.empty_like(x)
    raw.elementwise("axpby", x.contiguous(), y, z=z.contiguous(), alpha=alpha, beta=beta)
    return y


class _RevStack(torch.autograd.Function):
    """The residual streams (x1, x2) / (x, v) are carried in fp32 by default -- RevNet keeps no per-layer
    activations, so this costs two activation-sized buffers -- while every block F runs in the compute dtype.
    Reconstruction x1 = y2 - F(x2) is then exact to fp32 rounding instead of accumulating bf16 error over the depth.
    ``revnet_stream_dtype`` "calculation" keeps the RevNet streams in the compute dtype, as the reference does (its
    RevGradOp adds and subtracts in the activations' dtype, src/model/revnet.py:23,69): 4 instead of 10 bytes per
    element in every fused stream update (profiles/r6_revnet_stream.md)."""

    @staticmethod
    def forward(ctx, x, blocks: typing.List[Block], mode: str, alpha: float, calc: bool = False,
                gcalc: bool = False):
        """both streams start as the body input x; returns the body output y1 + y2 in x's dtype"""
        dt = x.dtype
        calc = calc and mode == "revnet"
        sd = _stream_dtype(dt, calc)
        x1 = x2 = _to_stream(x, sd)
        low = dt != sd                      # fused fp32 <- fp32 + bf16 kernels on the GPU
        with torch.no_grad():
            if calc:
                # streams in the compute dtype (the reference's RevGradOp): y2 = x1 + F(x2) from the block's last
                # GEMM's epilogue (F.StreamSink with a bf16 residual), else one elementwise add
                for f in blocks:
                    sink = _sink(x1, 1.0)
                    fx = f(x2, sink)
                    nx2 = sink.out if sink is not None and sink.out is not None else _add(x1, fx)
                    x1, x2 = x2, nx2
            elif mode == "revnet" and low:
                # the bf16 copy of the fp32 stream is the (bf16) input itself: bf16 -> fp32 -> bf16 is exact
                x2b = x.contiguous() if x.dtype == torch.bfloat16 else raw.to_bf16(x2)
                for f in blocks:
                    # y2 = x1 + F(x2) and its bf16 copy: from the block's last GEMM when it can take the update
                    # (F.StreamSink), else one mix_f32 pass
                    sink = _sink(x1, 1.0)
                    fx = f(x2b, sink)
                    if sink is not None and sink.out32 is not None:
                        nx2, nb = sink.out32, fx
                    else:
                        nb = torch.empty_like(x2b)
                        nx2 = raw.mix_f32(x1, fx, 1.0, 1.0, yb=nb)
                    x1, x2, x2b = x2, nx2, nb
            else:
                for f in blocks:
                    if mode == "revnet":
                        x1, x2 = x2, x1 + f(x2.to(dt)).to(sd)
                    else:  # momentum: (x, v) -> (x + v', v'), v' = a v + (1-a) F(x)
                        v = x2 * alpha + f(x1.to(dt)).to(sd) * (1.0 - alpha)
                        x1, x2 = x1 + v, v
        ctx.blocks, ctx.mode, ctx.alpha, ctx.dt, ctx.calc = blocks, mode, alpha, dt, calc
        # gradient streams in the compute dtype under fp32 activation streams (revnet_grad_stream_dtype)
        ctx.gcalc = gcalc and mode == "revnet" and not calc and dt == torch.bfloat16 and dt != _stream_dtype(dt)
        ctx.save_for_backward(x1, x2)
        return _sum_to(x1, x2, dt)

    @staticmethod
    def backward(ctx, g):
        y1, y2 = ctx.saved_tensors
        mode, alpha, dt = ctx.mode, ctx.alpha, ctx.dt
        sd = _stream_dtype(dt, ctx.calc)
        gd = dt if ctx.gcalc else sd
        g1 = g2 = g.to(gd).contiguous()     # d(y1 + y2): the same gradient reaches both streams
        y1b = g2b = None    # bf16 copies of y1 / g2, written by the previous block's fused fp32 mixes
        for f in reversed(ctx.blocks):
            if ctx.calc:
                # y1 = x2, y2 = x1 + F(x2), all in the compute dtype: the recomputed F's last GEMM writes
                # x1 = y2 - F(x2) (F.StreamSink, alpha -1) and the block's opening norm adds g1 into its dx
                # (F.GradSink); autograd still sees dL/dF = g2 for that last op
                sink = _sink(y2, -1.0)
                gsink = F.GradSink(g1) if sink is not None else None
                with torch.enable_grad():
                    x2 = y1.detach().requires_grad_(True)
                    fx = f(x2, sink, gsink)
                torch.autograd.backward(fx, g2)
                x1 = sink.out if sink is not None and sink.out is not None else _add(y2, fx.detach(), -1.0)
                if x2.grad is None:
                    dx2 = g1
                elif gsink is not None and gsink.fused:
                    # the norm's dx already holds g1; if another gradient reached x2 as well, autograd summed it in
                    dx2 = x2.grad
                else:
                    dx2 = _add(g1, x2.grad)
                y1, y2, g1, g2 = x1, y1, g2, dx2.contiguous()
                continue
            if ctx.gcalc:
                # fp32 activation streams (exact reconstruction x1 = y2 - F(x2) from the fused fp32 sink), bf16
                # gradient streams: the opening norm adds the bf16 g1 into its dx (F.GradSink with a bf16 R), and
                # dx2 / g2 stay bf16 -- the mixed-precision convention for activation gradients
                y1b = raw.to_bf16(y1) if y1b is None else y1b
                sink = _sink(y2, -1.0)
                gsink = F.GradSink(g1) if sink is not None else None
                with torch.enable_grad():
                    x2 = y1b.detach().requires_grad_(True)
                    fx = f(x2, sink, gsink)
                torch.autograd.backward(fx, g2)
                if sink is not None and sink.out32 is not None:
                    x1, nb1 = sink.out32, fx.detach()
                else:
                    nb1 = torch.empty_like(y1b)
                    x1 = raw.mix_f32(y2, fx.detach(), 1.0, -1.0, yb=nb1)
                if x2.grad is None:
                    dx2 = g1
                elif gsink is not None and gsink.fused:
                    dx2 = x2.grad            # the norm's dx already holds g1 (and anything else autograd summed in)
                else:
                    dx2 = _add(g1, x2.grad)
                y1b = nb1
                y1, y2, g1, g2 = x1, y1, g2, dx2.contiguous()
                continue
            if mode == "revnet":
                # y1 = x2, y2 = x1 + F(x2)
                bf = dt == torch.bfloat16
                if bf:
                    y1b = raw.to_bf16(y1) if y1b is None else y1b
                    g2b = raw.to_bf16(g2) if g2b is None else g2b
                # the recomputed F's last GEMM can also produce the reconstruction x1 = y2 - F(x2) (and its bf16
                # copy); its output is then that copy, and the backward below still receives dL/dF = g2 for it
                sink = _sink(y2, -1.0) if bf else None
                # and the norm opening the block can produce dx2 = g1 + dF/dx2 in fp32 with its bf16 copy
                gsink = F.GradSink(g1) if sink is not None else None
                with torch.enable_grad():
                    x2 = (y1b if bf else y1.to(dt)).detach().requires_grad_(True)
                    fx = f(x2, sink, gsink)
                torch.autograd.backward(fx, g2b if bf else g2.to(dt))
                if bf:
                    # x1 = y2 - F(x2) and dx2 = g1 + dF/dx2, each with its bf16 copy for the next (earlier) block
                    if sink is not None and sink.out32 is not None:
                        x1, nb1 = sink.out32, fx.detach()
                    else:
                        nb1 = torch.empty_like(y1b)
                        x1 = raw.mix_f32(y2, fx.detach(), 1.0, -1.0, yb=nb1)
                    if x2.grad is None:
                        dx2, nb2 = g1, None
                    elif gsink is not None and gsink.out32 is not None:
                        if x2.grad.data_ptr() == gsink.ptr:
                            dx2, nb2 = gsink.out32, x2.grad
                        else:   # another gradient reached x2 besides the norm's (or autograd copied it): x2.grad
                            # already holds g1 (summed in bf16) -- correct, at bf16 precision
                            dx2, nb2 = x2.grad.float(), x2.grad
                    else:
                        nb2 = torch.empty_like(y1b)
                        dx2 = raw.mix_f32(g1, x2.grad, 1.0, 1.0, yb=nb2)
                    y1b, g2b = nb1, nb2
                else:
                    x1 = y2 - fx.detach().to(sd)
                    dx2 = g1 if x2.grad is None else g1 + x2.grad.to(sd)
                y1, y2, g1, g2 = x1, y1, g2, dx2
            else:
                # y1 = x + v', y2 = v' ; v' = a v + (1-a) F(x)
                x = y1 - y2
                gv_tot = g2 + g1
                with torch.enable_grad():
                    xr = x.to(dt).detach().requires_grad_(True)
                    fx = f(xr)
                torch.autograd.backward(fx, (gv_tot * (1.0 - alpha)).to(dt))
                v = (y2 - fx.detach().to(sd) * (1.0 - alpha)) / alpha
                gx = g1 if xr.grad is None else g1 + xr.grad.to(sd)
                y1, y2, g1, g2 = x, v, gx, gv_tot * alpha
        # the body input fed both streams: its gradient is the sum, rounded once
        return _sum_to(g1, g2, dt), None, None, None, None, None


class _Checkpoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, f: Block):
        with torch.no_grad():
            y = f(x)
        ctx.f = f
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        with torch.enable_grad():
            xr = x.detach().requires_grad_(True)
            y = ctx.f(xr)
        torch.autograd.backward(y, dy)
        return xr.grad, None


def _calc_stream(builder: Builder) -> bool:
    v = str(getattr(builder.params, "revnet_stream_dtype", "float32"))
    if v not in ("float32", "calculation"):
        raise ValueError(f"revnet_stream_dtype must be 'float32' or 'calculation', not {v!r}")
    return v == "calculation"


def _calc_grad_stream(builder: Builder) -> bool:
    v = str(getattr(builder.params, "revnet_grad_stream_dtype", "float32"))
    if v not in ("float32", "calculation"):
        raise ValueError(f"revnet_grad_stream_dtype must be 'float32' or 'calculation', not {v!r}")
    return v == "calculation"


def run_body(builder: Builder, src: Act, strategy: str, configs, depth: int) -> Act:
    stack = builder.scope.snapshot()
    dims = src.dims
    blocks = [Block(builder, cfg, i, c, stack, dims) for i in range(depth) for c, cfg in enumerate(configs)]
    if builder.register or not torch.is_grad_enabled() or not src.t.requires_grad:
        # registration / inference: plain forward through the same blocks
        if strategy in ("revnet", "momentum"):
            dt = src.t.dtype
            sd = _stream_dtype(dt, strategy == "revnet" and _calc_stream(builder))
            x1 = x2 = src.t.to(sd)
            for f in blocks:
                if strategy == "revnet":
                    x1, x2 = x2, x1 + f(x2.to(dt)).to(sd)
                else:
                    a = builder.params.momentumnet_alpha
                    v = x2 * a + f(x1.to(dt)).to(sd) * (1.0 - a)
                    x1, x2 = x1 + v, v
            return Act((x1 + x2).to(dt), dims)
        x = src.t
        for f in blocks:
            x = f(x)
        return Act(x, dims)
    if strategy in ("revnet", "momentum"):
        y = _RevStack.apply(src.t, blocks, strategy, builder.params.momentumnet_alpha, _calc_stream(builder),
                            _calc_grad_stream(builder))
        return Act(y, dims)
    x = src.t
    for f in blocks:
        if strategy == "checkpoint":
            x = _Checkpoint.apply(x, f)
        else:
            x = f(x)
    return Act(x, dims)
