"""Every layer of the reference block grammar (``LAYER_FUNCTIONS``, src/model/frontend.py:58-75).

Each function takes ``BlockArgs`` and returns an ``Act``. Shapes come from the named-dim rules in ``dims.py``;
compute goes through ``ops.functional`` (HIP kernels on GPU). Two layers have fused fast paths that the hot
configs hit: ``feed_forward`` (act-in / linear-out, residual fused into the second GEMM epilogue) and
dot-product ``attention`` (in-linear, batched k/q/v GEMM, flash attention). Both create their variables in exactly
the order of the composable path, so checkpoints and init are identical whichever path runs.

Reference citations per layer are in the docstrings.
"""
from __future__ import annotations

import math
import string
import typing

import torch

from ..config import Dim, anonymize_dim, unanonymize_dim
from ..ops import aux as X
from ..ops import functional as F
from ..ops import raw as R
from ..parallel import state as pstate
from . import dims as D
from .context import Act, BlockArgs
from .variables import constant_init, fan_in_size, normal_init, orthogonal_init

ACTIVATIONS = ('relu', 'sigmoid', 'tanh', 'gelu', 'lecun_tanh', 'silu', 'mish', 'mtf_mish', 'softsign', 'exp')


# ================================================================================================================
# variables (ref src/model/backend.py:43-118)
def orthogonal_var(args: BlockArgs, dims: typing.List[Dim], fan_in_dims: typing.Optional[typing.List[Dim]] = None,
                   shard: typing.Optional[typing.Tuple[Dim, Dim]] = None):
    """shard = (local, global) dim: TP-split axis other than heads (tp_layout intermediate)"""
    p = args.params
    gb = args.builder
    fan_dims = None if fan_in_dims is None else gb._global_dims(list(fan_in_dims))
    if fan_dims is not None and shard is not None:
        fan_dims = [shard[1] if d == shard[0] else d for d in fan_dims]
    sbd = bool(p.scale_by_depth and args.is_last)

    def factory(gdims):
        return orthogonal_init([d.size for d in gdims], fan_in_size(fan_dims), sbd, p.depth)
    return args.builder.variable(args, "orthogonal_var", dims, factory, shard=shard)


def normal_var(args: BlockArgs, dims: typing.List[Dim], stddev: float = 0.02, mean: float = 0.):
    return args.builder.variable(args, "normal_var", dims, lambda gd: normal_init([d.size for d in gd], stddev, mean))


def constant_var(args: BlockArgs, dims: typing.List[Dim], value: float):
    return args.builder.variable(args, "constant_var", dims, lambda gd: constant_init([d.size for d in gd], value))


def _scoped(args: BlockArgs, name: str, fn, *a, **kw):
    with args.builder.scope(name):
        return fn(*a, **kw)


# ================================================================================================================
# named einsum (torch autograd) for the exotic paths; weights reached through it get .grad, folded afterwards
def named_einsum(inputs: typing.Sequence[Act], out_dims: typing.List[Dim]) -> Act:
    alld = []
    for a in inputs:
        for d in a.dims:
            if d not in alld:
                alld.append(d)
    for d in out_dims:
        if d not in alld:
            raise ValueError(f"output dim {d} not in inputs")
    pool = string.ascii_letters
    letters = {d: pool[i] for i, d in enumerate(alld)}
    eq = ",".join("".join(letters[d] for d in a.dims) for a in inputs) + "->" + "".join(letters[d] for d in out_dims)
    dt = inputs[0].t.dtype
    out = torch.einsum(eq, *[a.t.to(dt) for a in inputs])
    return Act(out, out_dims)


def rename(a: Act, old: Dim, new: Dim) -> Act:
    return Act(a.t, [new if d == old else d for d in a.dims])


def anonymize(a: Act, dim: Dim) -> Act:
    return rename(a, dim, anonymize_dim(dim))


# ================================================================================================================
# linear (ref backend.py:108-118, basic.py:33-34)
def linear(args: BlockArgs, old: typing.List[Dim], new: typing.List[Dim], act: typing.Optional[str] = None,
           sink=None, relu_grad=None) -> Act:
    x = args.tensor
    w = _scoped(args, "linear", orthogonal_var, args, list(old) + list(new), list(old))
    wdims = D.deduplicate(list(old) + list(new))
    odims = D.deduplicate(D.subtract(x.dims, old) + list(new))
    try:
        plan = F.linear_plan(tuple(x.dims), tuple(wdims), tuple(odims))
    except (NotImplementedError, ValueError):
        plan = None
    tp = pstate.tp_size() > 1
    if plan is not None:
        if act and plan.row_parallel and tp:   # all-reduce must precede the activation
            y = F.activation(F.linear(x.t, w, x.dims, wdims, odims), act)
        else:
            y = F.linear(x.t, w, x.dims, wdims, odims, act=act, sink=sink, relu_grad=relu_grad)
        return Act(y, odims)
    hd = args.params.head_dim
    xt = x.t
    if tp and hd in wdims and hd not in x.dims:
        xt = F.tp_copy(xt)                    # column-parallel: all-reduce dX in backward
    y = named_einsum([Act(xt, x.dims), Act(w, wdims)], odims).t
    if tp and hd in x.dims and hd in wdims and hd not in odims:
        y = F.tp_reduce(y)                    # row-parallel: all-reduce the partial sums
    return Act(F.activation(y, act), odims)


def linear_to_features(args: BlockArgs, old: typing.List[Dim]) -> Act:
    return linear(args, old, args.params.feature_dims)


def linear_from_features(args: BlockArgs, new: typing.List[Dim]) -> Act:
    return linear(args, args.params.feature_dims, new)


def wrapped_linear(args: BlockArgs) -> Act:
    old, new = D.linear_shapes(args.params, args, args.tensor.dims)
    return linear(args, old, new)


def _activation_name(args: BlockArgs) -> typing.Optional[str]:
    for a in args:
        if a in ACTIVATIONS:
            return a
    return None


def activate(args: BlockArgs) -> Act:
    """ref src/model/activation.py:201-211 -- first known activation in the extras; identity otherwise."""
    name = _activation_name(args)
    x = args.tensor
    if name is None:
        return x
    if name == "mtf_mish":
        name = "mish"
    return Act(F.activation(x.t, name), x.dims)


def dropout(args: BlockArgs) -> Act:
    """ref basic.py:25-30 (`dropout_rate<x>` extra)."""
    keep = 1.0
    for extra in args:
        if extra.startswith('dropout_rate'):
            keep = 1 - float(extra[len('dropout_rate'):])
    x = args.tensor
    if keep >= 1.0 or not args.builder.train:
        return x
    return Act(F.dropout(x.t, keep, args.builder.next_dropout_seed()), x.dims)


def rezero(args: BlockArgs) -> Act:
    """ref basic.py:21-22: x * g, g initialised to 0."""
    g = _scoped(args, "rezero", constant_var, args, [], 0.0)
    x = args.tensor
    return Act(F.rezero(x.t, g), x.dims)


def mixture_of_experts(args: BlockArgs) -> Act:
    """ref basic.py:37-44: dense soft mixture, gate = softmax_experts(x Wg), out = sum_e gate_e * x W_e."""
    p = args.params
    old, new = D.linear_shapes(p, args, args.tensor.dims)
    gate = linear(args, old, [p.expert_dim])
    w = _scoped(args, "moe", orthogonal_var, args, list(old) + list(new) + [p.expert_dim])
    wdims = D.deduplicate(list(old) + list(new) + [p.expert_dim])
    odims = D.deduplicate(D.subtract(args.tensor.dims, old) + list(new))
    x = args.tensor
    rest = D.subtract(x.dims, old)
    T, K, N, E = D.size(rest), D.size(old), D.size(new), p.expert_dim.size
    if (list(x.dims) == rest + list(old) and list(gate.dims) == rest + [p.expert_dim] and odims == rest + list(new)
            and wdims == list(old) + list(new) + [p.expert_dim] and pstate.tp_size() == 1 and X.moe_ok(x.t, E, K)):
        # one GEMM over the expert-minor weight + the fused softmax / expert contraction kernel (K15)
        y = X.moe(x.t, gate.t, w, T, K, N, E)
        return Act(y.view([d.size for d in odims]), odims)
    g = gate.t.float()
    ei = gate.dims.index(p.expert_dim)
    g = torch.softmax(g - g.amax(ei, keepdim=True).detach(), ei).to(args.tensor.t.dtype)
    return named_einsum([args.tensor, Act(g, gate.dims), Act(w, wdims)], odims)


def activated_linear(args: BlockArgs, prefix: str) -> Act:
    """ref basic.py:47-57."""
    # (only an out-projection can be a block's last product)
    sink = getattr(args, "stream_sink", None) if prefix == 'out:' else None
    args = args([a[len(prefix):] for a in args if a.startswith(prefix)])
    ff = mixture_of_experts if 'mixture_of_experts' in args else wrapped_linear
    act = _activation_name(args)
    if sink is not None and ff is wrapped_linear and act is None and _plain(list(args)):
        # the block's last product: the RevNet stream update rides in its epilogue (F.StreamSink)
        old, new = D.linear_shapes(args.params, args, args.tensor.dims)
        return linear(args, old, new, sink=sink)
    # a relu product straight into a norm: the norm's backward applies relu' (F.ReluGrad)
    rg = (F.ReluGrad() if act == "relu" and 'norm' in args and _plain([a for a in args if a != 'norm'])
          else None)
    if ff is wrapped_linear and act is not None and act != "mtf_mish":
        old, new = D.linear_shapes(args.params, args, args.tensor.dims)
        out = linear(args, old, new, act=act, relu_grad=rg)   # activation fused into the GEMM epilogue
    else:
        rg = None
        out = activate(args(ff(args)))
    out = dropout(args(out))
    if 'glu' in args or 'glu_add' in args:
        gate = ff(args)
        out = Act(X.glu(out.t, gate.t), out.dims)
    if 'glu_add' in args:
        extra = activate(args(ff(args)))
        out = Act(F.add(out.t, extra.t), out.dims)
    if 'norm' in args:
        out = norm(args(out), relu_grad=rg)
    return out


def activated_linear_in(args: BlockArgs) -> Act:
    return activated_linear(args, 'in:')


def activated_linear_out(args: BlockArgs) -> Act:
    return activated_linear(args, 'out:')


def _plain(extras: typing.List[str]) -> bool:
    """no glu/glu_add/norm/moe/dropout in this linear's extras (the fused fast paths' precondition)"""
    for e in extras:
        if e in ('glu', 'glu_add', 'norm', 'mixture_of_experts', 'mtf_mish') or e.startswith('dropout_rate'):
            return False
    return True


# ================================================================================================================
# feed_forward (ref basic.py:68-69) with the fused fast path
def feed_forward(args: BlockArgs) -> Act:
    p = args.params
    ins = [a[3:] for a in args if a.startswith('in:')]
    outs = [a[4:] for a in args if a.startswith('out:')]
    x = args.tensor
    act_in = next((a for a in ins if a in ACTIVATIONS), None)
    act_out = next((a for a in outs if a in ACTIVATIONS), None)
    if _plain(ins) and _plain(outs) and act_out is None and act_in != "mtf_mish":
        a_in = args(ins)
        old1, new1 = D.linear_shapes(p, a_in, x.dims)
        mdims = D.deduplicate(D.subtract(x.dims, old1) + list(new1))
        a_out = args(outs)
        old2, new2 = D.linear_shapes(p, a_out, mdims)
        odims = D.deduplicate(D.subtract(mdims, old2) + list(new2))
        try:
            p1 = F.linear_plan(tuple(x.dims), tuple(D.deduplicate(old1 + new1)), tuple(mdims))
            p2 = F.linear_plan(tuple(mdims), tuple(D.deduplicate(old2 + new2)), tuple(odims))
            ok = p1.x_perm is None and p1.o_perm is None and p2.x_perm is None and p2.o_perm is None
        except (NotImplementedError, ValueError):
            ok = False
        tp = pstate.tp_size()
        if (ok and tp > 1 and p.tp_layout == "intermediate" and list(old1) == list(p.feature_dims)
                and list(new1) == list(p.intermediate) and len(new1) == 1 and list(old2) == list(new1)
                and list(new2) == list(p.feature_dims) and new1[0].size % tp == 0 and x.dims[2:] == old1):
            # intermediate axis split over TP: same variables and global shapes as the heads layout,
            # sharded along the intermediate instead of the heads (checkpoints reshard between the two)
            hg = args.builder.global_params.head_dim
            ig = new1[0]
            il = Dim(ig.name, ig.size // tp)
            w1 = _scoped(a_in, "linear", orthogonal_var, a_in, [hg, p.key_dim, il], [hg, p.key_dim], shard=(il, ig))
            w2 = _scoped(a_out, "linear", orthogonal_var, a_out, [il, hg, p.key_dim], [il], shard=(il, ig))
            xg = list(x.dims[:2]) + [hg, p.key_dim]
            res = args.residual if (args.residual is not None and args.residual.dims == odims) else None
            y = F.ffn_itp(x.t, w1, w2, xg, [hg, p.key_dim, il], list(x.dims[:2]) + [il], [il, hg, p.key_dim], xg,
                          act_in, residual=res.t if res is not None else None,
                          carrier=getattr(args, "residual_carrier", None) if res is not None else None)
            if res is not None:
                args.residual_consumed = True
            return Act(y, odims)
        if ok:
            w1 = _scoped(a_in, "linear", orthogonal_var, a_in, list(old1) + list(new1), list(old1))
            w2 = _scoped(a_out, "linear", orthogonal_var, a_out, list(old2) + list(new2), list(old2))
            res = args.residual if (args.residual is not None and args.residual.dims == odims) else None
            y = F.ffn(x.t, w1, w2, x.dims, D.deduplicate(old1 + new1), mdims, D.deduplicate(old2 + new2), odims,
                      act_in, residual=res.t if res is not None else None,
                      carrier=getattr(args, "residual_carrier", None) if res is not None else None)
            if res is not None:
                args.residual_consumed = True
            return Act(y, odims)
    return activated_linear_out(args(activated_linear_in(args)))


def group_linear(args: BlockArgs) -> Act:
    """ref basic.py:72-74: per-head block-diagonal linear."""
    p = args.params
    new = [anonymize_dim(p.key_dim) if d == p.key_dim else d for d in p.feature_dims]
    out = linear(args('group'), p.feature_dims, new)
    # the reference reshapes back to the input shape; for a head-less input (reduced_half_linear) that reshape is
    # size-inconsistent in the reference, so here the head dim is kept and `_features_per_head` renamed back
    return Act(out.t, [unanonymize_dim(d) if d.name == "_" + p.key_dim.name else d for d in out.dims])


def sum_heads(args: BlockArgs) -> Act:
    """ref basic.py:77-78 (X06: all-reduce over the TP group when heads are split)."""
    x = args.tensor
    hd = args.params.head_dim
    i = x.dims.index(hd)
    y = _TPSum.apply(X.sum_axis(x.t, i))
    return Act(y, [d for d in x.dims if d != hd])


class _TPSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return pstate.tp_all_reduce(x.clone())

    @staticmethod
    def backward(ctx, dy):
        return dy


def transpose_sequence_features(args: BlockArgs) -> Act:
    """ref basic.py:81-86 (needs features_per_head == sequence)."""
    p = args.params
    assert p.features_per_head == p.sequence_length, "ToDo: Support other shapes"
    x = args.tensor
    si = next(i for i, d in enumerate(x.dims) if d.name == "sequence")
    fi = x.dims.index(p.key_dim)
    return Act(X.swap_axes(x.t, si, fi), x.dims)


def reduced_half_linear(args: BlockArgs) -> Act:
    """ref basic.py:89-90."""
    return group_linear(args(sum_heads(args)))


def product_key_memory(args: BlockArgs) -> Act:
    """ref basic.py:93-115 (typo A6 fixed): product-key memory with top-1 per sub-key axis."""
    p = args.params
    x = args.tensor
    anon_key = anonymize_dim(p.key_dim)
    features = [p.pkm_dim, anon_key]
    old = D.linear_shapes(p, args, x.dims).old
    assign = linear(args, old, [p.head_dim] + features)
    assign = norm(args(assign), features)
    table = _scoped(args, "embed", normal_var, args, [p.product_key_value_dim] + list(p.feature_dims),
                    p.embedding_stddev)
    lead = [d for d in assign.dims if d not in (p.head_dim, p.pkm_dim, anon_key)]
    if (assign.dims[-3:] == [p.head_dim, p.pkm_dim, anon_key] and list(p.feature_dims) == [p.head_dim, p.key_dim]
            and X.product_key_ok(assign.t, table)):
        # fused top-1 / index combine + value-weighted gather kernels (K14)
        return Act(X.product_key(assign.t, table), lead + [p.head_dim, p.key_dim])
    a = assign.t.double()
    ki = assign.dims.index(anon_key)
    pi = assign.dims.index(p.pkm_dim)
    normalizer = a.amax(ki, keepdim=True).sum(pi, keepdim=True)
    a = torch.exp(a - normalizer.detach())
    nsum = a.sum(ki, keepdim=True).prod(pi, keepdim=True)
    val, idx = a.max(ki, keepdim=True)
    mult = (p.features_per_head ** torch.arange(p.pkm_axes, device=a.device)).view(
        [p.pkm_axes if i == pi else 1 for i in range(a.dim())])
    idx = (idx * mult).sum(pi, keepdim=True)
    val = val.prod(pi, keepdim=True) / nsum
    keep = [d for d in assign.dims if d not in (anon_key, p.pkm_dim)]
    idx = idx.reshape([d.size for d in keep])
    val = val.reshape([d.size for d in keep]).to(x.t.dtype)
    # gather per head: out[..., h, f] = table[idx[..., h], h, f]
    hi = keep.index(p.head_dim)
    flat_idx = idx.movedim(hi, -1)                                   # [..., h]
    gathered = table.permute(1, 0, 2)[torch.arange(p.head_dim.size, device=a.device), flat_idx]  # [..., h, f]
    out_dims = [d for d in keep if d != p.head_dim] + [p.head_dim, p.key_dim]
    out = gathered * val.movedim(hi, -1).unsqueeze(-1)
    return Act(out, out_dims)


def feed_forward_product_key_memory(args: BlockArgs) -> Act:
    return product_key_memory(args(activated_linear_in(args)))


def bottleneck_group_linear(args: BlockArgs) -> Act:
    """ref basic.py:122-126."""
    sink = getattr(args, "stream_sink", None)
    args = args(activated_linear_in(args))
    args.name_extras.extend(['group', 'mid:group', 'out:group'])
    args = args(activated_linear(args, 'mid:'))
    args.stream_sink = sink
    return activated_linear_out(args)


# ================================================================================================================
# norm (ref normalization.py:22-34)
# norms whose normalized dims are not x's trailing dims run the norm kernel on a permuted copy (False: the torch
# autograd path -- the CPU tests' reference for it)
NORM_ANY_LAYOUT = True


def norm(args: BlockArgs, feature_shape: typing.Optional[typing.List[Dim]] = None, relu_grad=None) -> Act:
    p = args.params
    x = args.tensor
    feature_shape = list(D.linear_shapes(p, args, x.dims).old if feature_shape is None else feature_shape)
    group = 'group' in args
    normalized = [d for d in feature_shape if not (group and d == p.head_dim)]
    scale = _scoped(args, "norm", normal_var, args, feature_shape, 0.02, 1.0) if 'scale' in args else None
    shift = _scoped(args, "norm", normal_var, args, feature_shape, 0.02, 0.0) if 'shift' in args else None
    # fast path: normalized dims are the trailing dims of x; the param shape covers [groups] + normalized
    n = len(normalized)
    trailing = x.dims[-n:] == normalized
    grouped_ok = (not group) or (p.head_dim in feature_shape and x.dims[-n - 1] == p.head_dim and
                                 feature_shape == [p.head_dim] + normalized)
    if trailing and grouped_ok and (feature_shape == normalized or group):
        Fsz = int(math.prod(d.size for d in normalized))
        groups = p.head_dim.size if group else 1
        tp_stats = (not group) and p.head_dim in normalized and pstate.tp_size() > 1
        act = getattr(args, "fused_act", None) if not tp_stats else None
        y = F.norm(x.t, scale, shift, Fsz, groups, tp_stats=tp_stats,
                   carrier=getattr(args, "norm_carrier", None), grad_sink=getattr(args, "grad_sink", None), act=act,
                   relu_grad=relu_grad)
        args.fused_act_done = act is not None   # the frontend then skips the activation layer's own pass
        return Act(y, x.dims)
    # any other layout: permute to [others..., group?, normalized...] (row % groups = the group index), the same
    # kernel, permute back; parameters are permuted copies to [group?, normalized...] (their gradients flow back
    # through autograd instead of the fused main-grad accumulation)
    gdim = [p.head_dim] if group and p.head_dim in feature_shape and p.head_dim in x.dims else []
    if NORM_ANY_LAYOUT and all(d in x.dims for d in normalized) and (not group or gdim):
        others = [d for d in x.dims if d not in normalized and d not in gdim]
        order = others + gdim + normalized
        perm = [x.dims.index(d) for d in order]
        xp = x.t.permute(perm).contiguous()
        pshape = gdim + normalized

        def _param(t):
            if t is None:
                return None
            return t.permute([feature_shape.index(d) for d in pshape]).contiguous() if feature_shape != pshape else t
        Fsz = int(math.prod(d.size for d in normalized))
        groups = p.head_dim.size if gdim else 1
        tp_stats = (not gdim) and p.head_dim in normalized and pstate.tp_size() > 1
        y = F.norm(xp, _param(scale), _param(shift), Fsz, groups, tp_stats=tp_stats)
        inv = [order.index(d) for d in x.dims]
        return Act(y.view([d.size for d in order]).permute(inv), x.dims)
    # general path (torch autograd)
    axes = [x.dims.index(d) for d in normalized]
    xt = x.t.float()
    xt = xt - xt.mean(axes, keepdim=True)
    xt = xt * torch.rsqrt((xt * xt).mean(axes, keepdim=True) + 1e-5)
    out = Act(xt.to(x.t.dtype), x.dims)
    if scale is not None:
        out = named_einsum([out, Act(scale, feature_shape)], x.dims)
    if shift is not None:
        sh = named_einsum([Act(torch.ones_like(out.t), x.dims), Act(shift, feature_shape)], x.dims)
        out = Act(out.t + sh.t, x.dims)
    return out


def activation_layer(args: BlockArgs) -> Act:
    return activate(args)


# ================================================================================================================
# spatial mixing (ref spatial.py)
def _masked_map(args: BlockArgs) -> typing.Tuple[Act, typing.Optional[torch.Tensor]]:
    p = args.params
    dim = D.get_attention_dim(p, args.tensor.dims).dim
    tmp = anonymize_dim(dim)
    bias = embed(args, [p.head_dim, dim, tmp])
    mask = None
    if D.is_masked(p, args.tensor.dims):
        r = torch.arange(dim.size, device=bias.t.device)
        mask = (r.view(-1, 1) >= r.view(1, -1)).to(bias.t.dtype)   # [dim, tmp]: key <= query
    return bias, mask


def _apply_mask(bias: Act, mask, dim: Dim, tmp: Dim) -> Act:
    if mask is None:
        return bias
    return named_einsum([bias, Act(mask, [dim, tmp])], bias.dims)


def _cumsum_any(args: BlockArgs, mean: bool) -> Act:
    x = args.tensor
    dim = D.get_attention_dim(args.params, x.dims).dim
    axis = x.dims.index(dim)
    kv = args.builder.kv
    if kv is not None and axis == 1 and x.dims[0].name == "batch":
        # incremental decoding: the running fp32 sums of every position are kept; a decode step adds the new
        # token's input to the sum at pos - 1
        key = ("c", kv.cidx)
        kv.cidx += 1
        if kv.mode == "prefill":
            kv.keep_state(key, csum=torch.cumsum(x.t.float(), 1))
            return Act(F.cumsum(x.t, axis, mean=mean), x.dims)
        return Act(F.cumsum_step(x.t, kv.states[key]["csum"], kv.pos, mean), x.dims)
    if kv is not None:
        kv.unsupported = True
    return Act(F.cumsum(x.t, axis, mean=mean), x.dims)


def cumsum(args: BlockArgs) -> Act:
    """ref spatial.py:26-34."""
    return _cumsum_any(args, False)


def cummean(args: BlockArgs) -> Act:
    """ref spatial.py:37-39."""
    return _cumsum_any(args, True)


def _mixer_kv(args: BlockArgs, kv, x: Act, dim: Dim, tmp: Dim, causal: bool) -> Act:
    """the learned token mixer under incremental decoding: the prefill keeps the mixer input [B, S, H, F] and the
    masked weight; a decode step writes the new token's input at pos[b] and computes output row pos[b] only,
    y[b, h] = W[h, pos[b], :] · X[b, :, h] (one M = 1 GEMM batched over batch x heads)"""
    p = args.params
    i = kv.idx
    kv.idx += 1
    if kv.mode == "prefill":
        bias = embed(args, [p.head_dim, dim, tmp])
        w = bias.t.detach()
        wm = torch.tril(w) if causal else w.contiguous()
        kv.keep_state(i, x=x.t.contiguous(), w=wm)
        return Act(F.token_mixer(x.t, bias.t, causal), x.dims)
    st = kv.states[i]
    full = Dim(dim.name, st["x"].shape[1])
    embed(args, [p.head_dim, full, anonymize_dim(full)])   # the same variable bookkeeping as the prefill
    return Act(F.token_mixer_step(x.t, st["x"], st["w"], kv.pos), x.dims)


# the composable attention path runs its softmax / map variants on the flash kernels (False: the generic named-einsum
# path with materialised logits -- the CPU tests' reference for the routing)
FLASH_MAPS = True


def _attention_fast_ok(args: BlockArgs, ins, outs) -> bool:
    p = args.params
    x = args.tensor
    bad = ('embedded', 'positional', 'biased_softmax', 'biased_attention_map', 'scale_attention_map',
           'shared_key_value', 'input_as_value', 'group')
    if 'dot_product' not in args or 'context' not in args or any(b in args for b in bad):
        return False
    if not (_plain(ins) and _plain(outs)) or any(a in ACTIVATIONS for a in outs):
        return False
    if len(x.dims) != 4 or x.dims[2:] != list(p.feature_dims) or x.dims[1].name != "sequence":
        return False
    if D.get_attention_dim(p, x.dims).dim != x.dims[1]:
        return False
    return True


def _attention_kv(kv, x: Act, w_in, ws, w_in_dims, base_dims, w_out_dims, act_in, scale: float) -> Act:
    """causal dot-product attention with a KV cache (serving): prefill keeps k / v of the whole context; a decode
    step appends the new token's k / v and attends its query over the row's prefix in one kernel"""
    base = F.linear(x.t, w_in, x.dims, w_in_dims, base_dims, act=act_in)
    k, q, v = (F.linear(base, w, base_dims, w_out_dims, x.dims).contiguous() for w in ws)
    i = kv.idx
    kv.idx += 1
    if kv.mode == "prefill":
        kv.keep(i, k, v, scale)          # the scale may depend on the context length (attention_scale "sequence")
        return Act(F.attention_core(q, k, v, scale, True), x.dims)
    K, V, scale = kv.layers[i]
    B, S, H, Dh = K.shape
    o = torch.empty_like(q)
    R.decode_attn(q, k, v, K, V, o, kv.pos, B, S, H, Dh, scale)
    return Act(o, x.dims)


class _Fold:
    """[d0, ..., dim, ..., heads, fph] -> [B', S, heads, fph] with the attention dim second and every other spatial
    dim folded into the batch, so attention over a non-sequence axis (video ``three_axes``: height / width; ref
    ``src/utils_mtf.py:418-422`` cycles the attention dim) runs on the same flash kernels as sequence attention.
    Identity (no copy) when the attention dim already is dims[1] of a 4-d tensor."""

    def __init__(self, dims, dim: Dim, feat):
        lead = list(dims[:-len(feat)])
        self.ai = lead.index(dim)
        self.nlead = len(lead)
        self.order = [i for i in range(self.nlead) if i != self.ai] + [self.ai] + \
            list(range(self.nlead, len(dims)))
        self.perm_shape = [dims[i].size for i in self.order]
        self.identity = self.order == list(range(len(dims))) and self.nlead == 2
        self.B = int(math.prod(d.size for i, d in enumerate(lead) if i != self.ai))
        self.S = dim.size
        self.feat = [d.size for d in feat]
        self.inv = [self.order.index(i) for i in range(len(dims))]

    def fwd(self, t: torch.Tensor) -> torch.Tensor:
        if self.identity:
            return t
        return t.permute(self.order).reshape([self.B, self.S] + self.feat).contiguous()

    def back(self, t: torch.Tensor) -> torch.Tensor:
        if self.identity:
            return t
        return t.reshape(self.perm_shape).permute(self.inv).contiguous()


def _fold_of(p, dims, dim: Dim) -> typing.Optional[_Fold]:
    feat = list(p.feature_dims)
    if len(feat) != 2 or feat[0] != p.head_dim or list(dims[-2:]) != feat or dims[0].name != "batch":
        return None
    if dim not in dims[1:-2]:
        return None
    return _Fold(dims, dim, feat)


def _mixer_fast_ok(args: BlockArgs, x: Act, dim: Dim) -> bool:
    """the learned causal token mixer (biased_attention_map on the input as value) as one batched GEMM (K03)"""
    p = args.params
    if 'biased_attention_map' not in args or 'input_as_value' not in args:
        return False
    if any(k in args for k in ('dot_product', 'biased_softmax', 'scale_attention_map')):
        return False
    return (len(x.dims) == 4 and x.dims[0].name == "batch" and x.dims[1] == dim and
            x.dims[2:] == list(p.feature_dims))


def _note_mixer(args: BlockArgs, dim: Dim, causal: bool, before) -> None:
    """FLOP meter (models/model.py:count_flops_per_token): one token-mixer application costs 2 x features x (mixed
    positions) FLOPs per token forward, 3x that for training -- not 6 x its weight, which depth-shared mixers reuse
    at every application. Recorded once per application during the register pass."""
    if before is None:
        return
    store = args.builder.store
    n_t = (dim.size + 1) / 2 if causal else dim.size
    store.mixer_flops = getattr(store, "mixer_flops", 0.0) + 3 * 2 * args.params.features * n_t
    store.mixer_vars = getattr(store, "mixer_vars", set()) | (set(store.specs) - before)


def attention(args: BlockArgs) -> Act:
    """ref spatial.py:42-81 (all variants). Fast path: dot_product + context (causal flash attention)."""
    p = args.params
    p.attention_idx += 1
    x = args.tensor
    ins = [a[3:] for a in args if a.startswith('in:')]
    outs = [a[4:] for a in args if a.startswith('out:')]
    dim = D.get_attention_dim(p, x.dims).dim
    tmp = anonymize_dim(dim)
    if p.attention_scale == "sequence":
        scale = dim.size ** -0.5      # quirk A1 (spatial.py:60)
    else:
        scale = p.key_dim.size ** -0.5
    causal = D.is_masked(p, x.dims)

    if _attention_fast_ok(args, ins, outs):
        a_in = args(ins)
        act_in = next((a for a in ins if a in ACTIVATIONS), None)
        old1, new1 = D.linear_shapes(p, a_in, x.dims)
        base_dims = D.deduplicate(D.subtract(x.dims, old1) + list(new1))
        a_out = args(outs)
        old2, new2 = D.linear_shapes(p, a_out, base_dims)
        w_in = _scoped(a_in, "linear", orthogonal_var, a_in, list(old1) + list(new1), list(old1))
        ws = [_scoped(a_out, "linear", orthogonal_var, a_out, list(old2) + list(new2), list(old2)) for _ in range(3)]
        kv = args.builder.kv
        if kv is not None and causal and pstate.tp_size() == 1:
            return _attention_kv(kv, x, w_in, ws, D.deduplicate(old1 + new1), base_dims, D.deduplicate(old2 + new2),
                                 act_in, scale)
        res = args.residual if (args.residual is not None and args.residual.dims == x.dims) else None
        geo = (x.dims[0].size, x.dims[1].size, p.head_dim.size, p.key_dim.size)
        try:
            y = F.dot_attention(x.t, w_in, ws[0], ws[1], ws[2], x.dims, D.deduplicate(old1 + new1), base_dims,
                                D.deduplicate(old2 + new2), act_in, scale, causal, geo,
                                residual=res.t if res is not None else None,
                                carrier=getattr(args, "residual_carrier", None) if res is not None else None)
            if res is not None:
                args.residual_consumed = True
            return Act(y, x.dims)
        except NotImplementedError:
            pass

    if _mixer_fast_ok(args, x, dim):
        kv = args.builder.kv
        if kv is not None and causal:
            return _mixer_kv(args, kv, x, dim, tmp, causal)
        before = set(args.builder.store.specs) if args.builder.register else None
        bias = embed(args, [p.head_dim, dim, tmp])
        _note_mixer(args, dim, causal, before)
        return Act(F.token_mixer(x.t, bias.t, causal, sink=getattr(args, "stream_sink", None)), x.dims)
    fold = _fold_of(p, x.dims, dim) if FLASH_MAPS else None
    if (fold is not None and not fold.identity and args.builder.kv is None and 'biased_attention_map' in args
            and 'input_as_value' in args and not any(k in args for k in ('dot_product', 'biased_softmax',
                                                                           'scale_attention_map'))):
        # the learned token mixer over a non-sequence axis: the same K03 kernel on the folded input
        before = set(args.builder.store.specs) if args.builder.register else None
        bias = embed(args, [p.head_dim, dim, tmp])
        _note_mixer(args, dim, causal, before)
        return Act(fold.back(F.token_mixer(fold.fwd(x.t), bias.t, causal)), x.dims)
    if args.builder.kv is not None:
        args.builder.kv.unsupported = True     # the composable path below has no incremental form

    base = None
    if 'dot_product' in args or 'input_as_value' not in args:
        base = activated_linear_in(args)
    logit = None
    val = None
    key = None
    if 'dot_product' in args:
        if 'embedded' in args or 'context' in args:
            key = activated_linear_out(args(base))
        if 'embedded' in args or 'positional' in args:
            pe = embed(args, [dim] + list(p.feature_dims))
            key = pe if key is None else Act(key.t + _bcast(pe, key).t, key.dims)
        qry = activated_linear_out(args(base))
        qry = Act(qry.t * scale, qry.dims)
        if key is None:
            raise ValueError("dot_product attention needs 'context', 'embedded' or 'positional'")
        # flash core over [batch, seq, heads, fph] for every map combination (no [B, S, heads, S] logits):
        #   biased_softmax       -> additive [heads, S, S] map inside the softmax (attn_map kernels)
        #   scale_attention_map  -> multiplicative map on the probabilities (attn_map kernels)
        #   biased_attention_map -> (P + Bm) V = P V + Bm V: the learned token mixer (K03) on the same values
        # positional-only keys ([seq, heads, fph]) are broadcast over the batch
        quirk_a19 = 'shared_key_value' in args and not p.shared_key_value_mixing
        fold = _fold_of(p, x.dims, dim) if FLASH_MAPS and not quirk_a19 else None
        kdims_pos = [dim] + list(x.dims[-2:])   # positional-only keys: [attention dim, heads, fph]
        if fold is not None and qry.dims == x.dims and (key.dims == x.dims or key.dims == kdims_pos):
            # maps created in the order of the generic path below (variable scopes / checkpoint names)
            sb = _masked_map(args)[0] if 'biased_softmax' in args else None
            ab = _masked_map(args) if 'biased_attention_map' in args else None
            sc = _masked_map(args) if 'scale_attention_map' in args else None
            v = key if 'shared_key_value' in args else (
                Act(x.t, x.dims) if 'input_as_value' in args else activated_linear_out(args(base)))
            kt = fold.fwd(key.t) if key.dims == x.dims else key.t.unsqueeze(0).expand(fold.B, *key.t.shape)
            vt = fold.fwd(v.t) if v.dims == x.dims else v.t.unsqueeze(0).expand(fold.B, *v.t.shape)
            qt = fold.fwd(qry.t)
            cm = _apply_mask(sc[0], sc[1], dim, tmp).t if sc is not None else None
            if sb is None and cm is None:
                o = F.attention_core(qt, kt, vt, 1.0, causal)
            else:
                o = F.attention_map(qt, kt, vt, sb.t if sb is not None else None, cm, 1.0, causal)
            if ab is not None:
                bm = _apply_mask(ab[0], ab[1], dim, tmp).t
                if cm is not None:
                    bm = bm * cm
                o = o + F.token_mixer(vt.contiguous(), bm, causal)
            return Act(fold.back(o), x.dims)
        old = D.linear_shapes(p, args, x.dims).old
        logit_dims = D.subtract(x.dims, D.subtract(old, [p.head_dim])) + [tmp]
        logit = named_einsum([qry, anonymize(key, dim)], logit_dims)
        if 'shared_key_value' in args:
            # V = K attention. The reference keeps the key un-anonymised here (spatial.py:63-64 + :81), so its final
            # einsum does not contract over keys and yields rowsum(logit) * key_q -- no mixing at all (quirk A19).
            # Fixed by default (shared_key_value_mixing, docs/PARITY.md; the flash route above agrees); with the
            # switch off the reference's einsum is reproduced for checkpoints trained with it
            full = key if key.dims == x.dims else Act(key.t.unsqueeze(0).expand(x.dims[0].size, *key.t.shape),
                                                      x.dims)
            val = anonymize(full, dim) if p.shared_key_value_mixing else full
    if 'biased_softmax' in args:
        bias, mask = _masked_map(args)
        b = _apply_mask(bias, mask, dim, tmp)
        logit = Act(logit.t + _bcast(b, logit).t, logit.dims)
    if logit is not None:
        lt = logit.t.float()
        if causal:
            r = torch.arange(dim.size, device=lt.device)
            m = (r.view(-1, 1) < r.view(1, -1))  # key > query
            di, ti = logit.dims.index(dim), logit.dims.index(tmp)
            shape = [1] * lt.dim()
            shape[di], shape[ti] = dim.size, dim.size
            lt = lt.masked_fill(m.view(shape), float("-inf"))
        ti = logit.dims.index(tmp)
        lt = torch.softmax(lt, ti)
        logit = Act(lt.to(x.t.dtype), logit.dims)
    if 'biased_attention_map' in args:
        bias, mask = _masked_map(args)
        b = _apply_mask(bias, mask, dim, tmp)
        logit = b if logit is None else Act(logit.t + _bcast(b, logit).t, logit.dims)
    if 'scale_attention_map' in args:
        bias, mask = _masked_map(args)
        b = _apply_mask(bias, mask, dim, tmp)
        if logit is None:
            raise UserWarning(f"no spatial mixing with attention parameters {args.name_extras}")
        logit = Act(logit.t * _bcast(b, logit).t, logit.dims)
    if val is None:
        val = x if 'input_as_value' in args else activated_linear_out(args(base))
        val = anonymize(val, dim)
    if logit is None:
        raise UserWarning(f"no spatial mixing with attention parameters {args.name_extras}")
    return named_einsum([logit, val], x.dims)


def _bcast(a: Act, like: Act) -> Act:
    """broadcast `a` (subset dims) to `like`'s dim order"""
    t = a.t
    order = [d for d in like.dims if d in a.dims]
    t = t.permute([a.dims.index(d) for d in order])
    shape = [d.size if d in a.dims else 1 for d in like.dims]
    return Act(t.reshape(shape).expand([d.size for d in like.dims]), like.dims)


def convolution(args: BlockArgs) -> Act:
    """ref convolution.py:128-129: disabled in the reference."""
    raise ValueError("Convolution is currently broken")


# ================================================================================================================
# embeddings (ref embedding.py:174-231)
def _embed_var(args: BlockArgs, dims: typing.List[Dim]):
    if 'orthogonal' in args:
        return orthogonal_var(args, dims)
    return normal_var(args, dims, args.params.embedding_stddev)


def _relative(args: BlockArgs, shape: typing.List[Dim]) -> torch.Tensor:
    """ref RelativeEmbeddingForward (embedding.py:128-172): sinusoidal, no gradient."""
    p = args.params
    position_dims = D.subtract(D.subtract(shape, p.feature_dims), p.intermediate)
    feature_dims = D.linear_shapes(p, args, args.tensor.dims).old
    position_count = D.size(position_dims)
    cosine = 'cosine' in p.position_embedding
    dev = args.builder.device if not args.builder.register else "meta"
    # a constant of the shapes: generated once per (shape, features, dtype, device) and kept on the device (K11)
    cache = args.builder.__dict__.setdefault("_relative_cache", {})
    key = (tuple(shape), tuple(feature_dims), cosine, float(p.embedding_stddev), args.builder.dtype, str(dev))
    if key in cache:
        return cache[key]

    def multi_range(dims):
        sizes = [d.size for d in dims]
        out = torch.zeros(sizes, dtype=torch.float64, device="cpu")
        stride = 1
        for i, dsz in enumerate(sizes):
            shp = [1] * len(sizes)
            shp[i] = dsz
            out = out + (torch.arange(dsz, dtype=torch.float64) * stride).view(shp)
            stride *= dsz
        return out
    positions = multi_range(position_dims)
    features = multi_range(feature_dims)
    feature_count = D.size(feature_dims)
    additive = 0.
    if cosine:
        additive = torch.fmod(features, 2)
        features = (features - additive) / 2
        additive = additive * math.pi
        feature_count /= 2
    features = features + 4 / feature_count
    features = features - math.log(position_count / 2 / math.pi)
    features = torch.exp(features) + additive
    pl = "".join(string.ascii_lowercase[shape.index(d)] for d in position_dims)
    fl = "".join(string.ascii_lowercase[shape.index(d)] for d in feature_dims)
    sl = "".join(string.ascii_lowercase[i] for i in range(len(shape)))
    out = torch.einsum(f"{pl},{fl}->{sl}", positions, features)
    out = torch.sin(out) * p.embedding_stddev
    out = out.to(dtype=args.builder.dtype, device=dev)
    if str(dev) != "meta":
        cache[key] = out
    return out


# axial embeddings on the K12 kernel (False: the named-einsum product -- the CPU tests' reference)
AXIAL_KERNEL = True


def _embed(args: BlockArgs, shape: typing.List[Dim]) -> Act:
    p = args.params
    shape = list(shape)
    if 'absolute' in args:
        return Act(_embed_var(args, shape), shape)
    if 'axial' in args:
        splits = 2
        for a in args:
            if a.isdigit():
                splits = int(a)
                break
        position_dims = D.subtract(D.subtract(shape, p.feature_dims), p.intermediate)
        feature_dims = D.linear_shapes(p, args, args.tensor.dims).old
        tmp_dims, variables = [], []
        for dim in position_dims:
            base = int(dim.size ** (1 / splits))
            while dim.size % base != 0:
                base -= 1
            final = dim.size // base ** (splits - 1)
            for sz in [final] + [base] * (splits - 1):
                tdim = Dim(f'_{len(tmp_dims)}', sz)
                tmp_dims.append(tdim)
                variables.append(Act(_embed_var(args, [tdim] + list(feature_dims)), [tdim] + list(feature_dims)))
        if AXIAL_KERNEL and len(variables) <= 4:   # K12: the broadcast product in one kernel (fp32 factor grads)
            out_t = F.axial_embed([v.t for v in variables], int(math.prod(d.size for d in feature_dims)))
            return Act(out_t.reshape([d.size for d in shape]), shape)
        out = named_einsum(variables, tmp_dims + list(feature_dims))
        return Act(out.t.reshape([d.size for d in shape]), shape)
    if 'relative' in args:
        out = _relative(args, shape)
        if 'learned' in args:
            fd = D.linear_shapes(p, args, args.tensor.dims).old
            learned = _embed_var(args, fd)
            return named_einsum([Act(out, shape), Act(learned, fd)], shape)
        return Act(out, shape)
    raise ValueError("The following embeddings are supported: relative(-learned) or absolute(-split) or "
                     "axial(-split) are supported")


def embed(args: BlockArgs, shape: typing.List[Dim]) -> Act:
    with args.builder.scope("embed"):
        return _embed(args, shape)


def gather_embed(args: BlockArgs, shape: typing.List[Dim], idx: torch.Tensor, idx_dims: typing.List[Dim]) -> Act:
    """ref embedding.py:230-231: table [vocab, ...] gathered by integer indices."""
    with args.builder.scope("gather"):
        table = embed(args, shape)
    args.builder.last_gather_table = table.t
    V = shape[0].size
    Fsz = D.size(shape[1:])
    if table.t.dim() != 2:
        raise NotImplementedError("gather_embed over multi-dim rows")
    out = F.gather(idx, table.t, V, Fsz)
    return Act(out, list(idx_dims) + list(shape[1:]))


# ================================================================================================================
def split_path(args: BlockArgs) -> Act:
    """ref frontend.py:39-55: parallel branches separated by ';', combined by add or multiply."""
    from .frontend import run_layers
    base, *branches = '-'.join(args.name_extras).split(';')
    base = base.split('-')
    if 'add' in base:
        combine, out = "add", None
    elif 'multiply' in base:
        combine, out = "multiply", None
    else:
        raise ValueError("split_path needs 'add' or 'multiply'")
    for conf in branches:
        y, _ = run_layers(args.builder, conf.split(','), args.tensor)
        if out is None:
            out = y
        else:
            out = Act(F.add(out.t, y.t) if combine == "add" else out.t * y.t, out.dims)
    return out


LAYER_FUNCTIONS = {'feed_forward': feed_forward,
                   'attention': attention,
                   'cummean': cummean,
                   'cumsum': cumsum,
                   'norm': norm,
                   'rezero': rezero,
                   'activation': activation_layer,
                   'convolution': convolution,
                   'dropout': dropout,
                   'group_linear': group_linear,
                   'split_path': split_path,
                   'feed_forward_product_key_memory': feed_forward_product_key_memory,
                   'product_key_memory': product_key_memory,
                   'reduced_half_linear': reduced_half_linear,
                   'transpose_sequence_features': transpose_sequence_features,
                   'bottleneck_group_linear': bottleneck_group_linear,
                   'sum_heads': sum_heads}
