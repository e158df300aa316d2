"""Per-tensor optimizer in plain PyTorch: the exact reference semantics (src/optimizer/optimizers.py,
src/optimizer/__init__.py:31-66) and the oracle the fused HIP executor (optim/fused.py) is tested against.

Runs on CPU, and on GPU for chains the fused executor does not cover (``graft``).
"""
from __future__ import annotations

import math
import typing

import torch
import torch.distributed as dist

from ..parallel import state as pstate
from .chain import parse_chain


def opt_rsqrt(x: torch.Tensor) -> torch.Tensor:
    return 1.0 / torch.clamp(torch.sqrt(x), min=1e-5)


class TensorState:
    def __init__(self):
        self.slots: typing.Dict[str, torch.Tensor] = {}


class ReferenceOptimizer:
    def __init__(self, store, params):
        self.store = store
        self.params = params
        self.chain = parse_chain(params.optimizer)
        self.state: typing.Dict[str, TensorState] = {n: TensorState() for n in store.order}
        self.wd_mask = {n: store.specs[n].weight_decay_eligible(params) for n in store.order}

    # -- helpers --------------------------------------------------------------------------------------------------
    def _slot(self, name, key, like, shape=None):
        st = self.state[name].slots
        if key not in st:
            st[key] = torch.zeros(like.shape if shape is None else shape, dtype=torch.float32, device=like.device)
        return st[key]

    def _tp_sum(self, name, v: torch.Tensor) -> torch.Tensor:
        """scalar statistics of a TP-sharded tensor are summed over the TP group (X11/X12)"""
        if pstate.tp_size() > 1 and self.store.specs[name].tp_dim is not None:
            v = v.clone()
            pstate.tp_all_reduce(v)
        return v

    def _numel(self, name):
        s = self.store.specs[name]
        return s.numel * (pstate.tp_size() if s.tp_dim is not None else 1)

    # -- stages ---------------------------------------------------------------------------------------------------
    def _adam(self, name, g, ctx):
        b1, b2, sc = ctx["beta1"], ctx["beta2"], ctx["step_count"]
        v = self._slot(name, "exp_avg_p2", g)
        m = self._slot(name, "exp_avg_p1", g)
        v.mul_(b2).add_(g * g * (1 - b2))
        m.mul_(b1).add_(g * (1 - b1))
        return opt_rsqrt(v / (1 - b2 ** sc)) * m / (1 - b1 ** sc)

    def _sm3(self, name, g, ctx):
        if g.dim() == 0:
            return self._adam(name, g, ctx)
        accs = [self._slot(name, f"dim{i}", g, (g.shape[i],)) for i in range(g.dim())]
        shp = lambda i: [g.shape[i] if j == i else 1 for j in range(g.dim())]  # noqa: E731
        nu = accs[0].view(shp(0))
        for i in range(1, g.dim()):
            nu = torch.minimum(nu, accs[i].view(shp(i)))
        nu = nu + g * g
        spec = self.store.specs[name]
        for i, acc in enumerate(accs):
            red = [j for j in range(g.dim()) if j != i]
            new = nu.amax(dim=red) if red else nu.clone()
            if pstate.tp_size() > 1 and spec.tp_dim is not None and i != spec.tp_dim:
                dist.all_reduce(new, op=dist.ReduceOp.MAX, group=pstate.mesh().tp_group)   # X10
            acc.copy_(new)
        return g * opt_rsqrt(nu)

    def _novograd(self, name, g, ctx):
        if g.dim() == 0:
            return self._adam(name, g, ctx)
        b1, b2, sc = ctx["beta1"], ctx["beta2"], ctx["step_count"]
        p1 = self._slot(name, "exp_avg_p1", g)
        p2 = self._slot(name, "exp_avg_p2", g, ())
        p1.mul_(b1).add_(g * opt_rsqrt(p2))
        p2.mul_(b2).add_(self._tp_sum(name, (g * g).sum()) * (1 - b2))
        return b1 * p1 + g * opt_rsqrt(p2 / (1 - b2 ** sc))

    def _adafactor(self, name, g, ctx, arg=None):
        """Shazeer & Stern 2018: factored second moment over [rows = all leading dims, cols = last dim], update
        clipping d=1. Under TP the factored statistics are those of the FULL tensor: a sharded last dim leaves each
        rank partial row sums, a sharded leading dim partial column sums and a partial sum of the row factors --
        each is all-reduced over the TP group and divided by the global count."""
        sc = ctx["step_count"]
        b2 = float(arg) if arg else 1.0 - sc ** -0.8
        if g.dim() >= 2:
            rows = int(math.prod(g.shape[:-1]))
            cols = g.shape[-1]
            g2 = g.reshape(rows, cols)
            R = self._slot(name, "af_rows", g, (rows,))
            C = self._slot(name, "af_cols", g, (cols,))
            spec = self.store.specs[name]
            tp = pstate.tp_size()
            sharded = tp > 1 and spec.tp_dim is not None
            cols_sharded = sharded and spec.tp_dim == g.dim() - 1
            rows_sharded = sharded and not cols_sharded
            sq = g2 * g2
            rsum, csum = sq.sum(1), sq.sum(0)
            if cols_sharded:
                pstate.tp_all_reduce(rsum)
            if rows_sharded:
                pstate.tp_all_reduce(csum)
            ncols = cols * (tp if cols_sharded else 1)
            nrows = rows * (tp if rows_sharded else 1)
            R.mul_(b2).add_((rsum / ncols + 1e-30) * (1 - b2))
            C.mul_(b2).add_((csum / nrows + 1e-30) * (1 - b2))
            rtot = R.sum()
            if rows_sharded:
                rtot = rtot.clone()
                pstate.tp_all_reduce(rtot)
            vhat = R.view(-1, 1) * C.view(1, -1) / (rtot / nrows)
            u = (g2 * torch.rsqrt(torch.clamp(vhat, min=1e-30))).reshape(g.shape)
        else:
            v = self._slot(name, "af_v", g)
            v.mul_(b2).add_((g * g + 1e-30) * (1 - b2))
            u = g * torch.rsqrt(v)
        rms = torch.sqrt(self._tp_sum(name, (u * u).sum()) / self._numel(name))
        return u / torch.clamp(rms, min=1.0)

    # -- step -----------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, lr: float, step_count: int, grad_scale: float = 1.0):
        p = self.params
        ctx = {"beta1": p.opt_beta1, "beta2": p.opt_beta2, "step_count": float(step_count), "lr": lr}
        grads = {n: self.store.grad_view(n).float() * grad_scale for n in self.store.order
                 if self.store.specs[n].trainable}
        global_sq = None
        for name, g in grads.items():
            w = self.store.master_view(name)
            g = self.apply_chain(name, g, w, ctx, self.chain, grads, global_sq_ref=[global_sq])
            if self.store.specs[name].is_rezero:
                g = g * p.rezero_lr_multiplier
            if self.wd_mask[name] and p.weight_decay > 0:
                g = g + w * lr * p.weight_decay
            w.sub_(g)
        self.store.sync_compute()

    def apply_chain(self, name, g, w, ctx, chain, grads, global_sq_ref):
        for opt, args in chain:
            g = self.apply_stage(name, opt, args, g, w, ctx, grads, global_sq_ref)
        return g

    def apply_stage(self, name, opt, args, g, w, ctx, grads, global_sq_ref):
        if opt == "adam":
            return self._adam(name, g, ctx)
        if opt == "sm3":
            return self._sm3(name, g, ctx)
        if opt == "novograd":
            return self._novograd(name, g, ctx)
        if opt == "adafactor":
            return self._adafactor(name, g, ctx, args[0] if args else None)
        if opt == "momentum":
            mm, gm, nest = float(args[0]), float(args[1]), bool(int(args[2]))
            st = self._slot(name, "momentum", g)
            st.mul_(mm).add_(g * gm)
            return g + mm * st if nest else st.clone()
        if opt == "adaptive_clip":
            c = float(args[0])
            gn = torch.clamp(torch.rsqrt(self._tp_sum(name, (g * g).sum())), max=1e6)
            wn = torch.clamp(torch.sqrt(self._tp_sum(name, (w * w).sum())), min=1e-3)
            return g * torch.clamp(wn * gn * c, max=1.0)
        if opt == "l2norm_clip":
            c = float(args[0])
            return g * c * torch.rsqrt(torch.clamp(self._tp_sum(name, (g * g).sum()), min=c ** -2))
        if opt == "global_l2norm_clip":
            c = float(args[0])
            if global_sq_ref[0] is None:
                tot = sum(self._tp_sum(n, (gg * gg).sum()) for n, gg in grads.items())
                global_sq_ref[0] = torch.rsqrt(torch.clamp(tot, min=c ** -2))
            return g * c * global_sq_ref[0]
        if opt == "value_clip":
            c = float(args[0])
            return torch.clamp(g, -c, c)
        if opt == "gradient_centralisation":
            return g - self._tp_sum(name, g.sum()) / self._numel(name)
        if opt == "weight_centralisation":
            return g + self._tp_sum(name, w.sum()) / self._numel(name)
        if opt == "learning_rate":
            return g * ctx["lr"]
        if opt == "graft":
            inner, *iargs = args
            h = self.apply_stage(name, inner, tuple(iargs), g, w, ctx, grads, global_sq_ref)
            g2 = self._tp_sum(name, (g * g).sum())
            # an all-zero g gets a zero update (the reference's rsqrt(0) * 0 makes it NaN)
            return torch.where(g2 > 0, g * torch.rsqrt(g2.clamp(min=1e-38)), torch.zeros_like(g)) * \
                torch.sqrt(self._tp_sum(name, (h * h).sum()))
        raise ValueError(opt)

    # -- checkpoint -----------------------------------------------------------------------------------------------
    def state_dict(self) -> typing.Dict[str, torch.Tensor]:
        out = {}
        opt_str = self.params.optimizer.replace(':', '_')
        for name, st in self.state.items():
            for k, v in st.slots.items():
                out[f"{name}/{opt_str}/{k}"] = v   # ref slot naming src/optimizer/backend.py:23-25
        return out

    def named_slots(self) -> typing.Dict[str, torch.Tensor]:
        """every slot tensor under its reference name; slots are created lazily, so untouched ones are absent"""
        return self.state_dict()

    def load_state_dict(self, sd: typing.Dict[str, torch.Tensor]):
        opt_str = self.params.optimizer.replace(':', '_')
        for key, v in sd.items():
            name, rest = key.split(f"/{opt_str}/", 1)
            self.state[name].slots[rest] = v.clone().to(self.store.device)
