"""Block grammar: ``{"layer": ["name-extra-extra", ...], "skip": bool}`` (ref src/model/frontend.py:21-55).

Layers run sequentially inside the block's scope; ``skip`` adds the block input back for the ``none`` and
``checkpoint`` memory strategies. When the last layer has a fused fast path (feed_forward / dot-product attention)
the residual add is folded into its final GEMM / attention epilogue instead of a separate elementwise pass.
"""
from __future__ import annotations

import typing

from ..config import BlockConfig
from ..ops import functional as F
from .context import Act, BlockArgs, Builder
from .layers import LAYER_FUNCTIONS

_FUSABLE_LAST = ("feed_forward", "attention")


def run_layers(builder: Builder, layers: typing.List[str], x: Act, residual: typing.Optional[Act] = None,
               stream_sink=None, grad_sink=None) -> typing.Tuple[Act, bool]:
    out = x
    consumed = False
    seen: typing.Dict[str, int] = {}
    n = len(layers)
    # pre-norm block whose last layer takes the residual in its epilogue: that layer's residual gradient goes to
    # the opening norm (same input tensor x), which adds it inside its backward kernel (F.ResidualGrad)
    carrier = None
    if (residual is not None and residual is x and n > 1 and layers[0].split('-')[0] == "norm"
            and layers[-1].split('-')[0] in _FUSABLE_LAST):
        carrier = F.ResidualGrad()
    skip_act = False
    for idx, layer in enumerate(layers, 1):
        name, *extras = layer.split('-')
        if name not in LAYER_FUNCTIONS:
            raise ValueError(f"unknown layer {name!r}; known: {sorted(LAYER_FUNCTIONS)}")
        args = BlockArgs(builder, out, extras, idx == n)
        args.fn_name = name
        args.fn_occurrence = seen.get(name, 0)
        seen[name] = args.fn_occurrence + 1
        builder.shared.begin_layer((builder.config_idx, name, args.fn_occurrence))
        if idx == n and residual is not None and name in _FUSABLE_LAST:
            args.residual = residual
            args.residual_carrier = carrier
        if idx == 1 and carrier is not None:
            args.norm_carrier = carrier
        if idx == n and stream_sink is not None:
            args.stream_sink = stream_sink   # consumed (sink.out set) only by a layer that can fuse it
        if idx == 1 and grad_sink is not None and name == "norm":
            args.grad_sink = grad_sink       # the norm on the block input itself
        if name == "norm" and idx < n:
            args.fused_act = _fusable_act(layers[idx])
        with builder.scope(name + '_'):
            if skip_act:                     # applied by the preceding norm's kernel (variable-free layer)
                skip_act = False
            else:
                out = LAYER_FUNCTIONS[name](args)
        skip_act = getattr(args, "fused_act_done", False)
        consumed = consumed or getattr(args, "residual_consumed", False)
    return out, consumed


def _fusable_act(layer: str) -> typing.Optional[str]:
    """the activation of an `activation-<act>` layer that the norm kernels can apply (and differentiate) in place"""
    from ..ops import raw
    name, *extras = layer.split('-')
    if name != "activation":
        return None
    from .layers import ACTIVATIONS
    act = next((a for a in extras if a in ACTIVATIONS), None)
    return act if act in raw.ACTS and raw.ACTS[act] != 0 else None


def block_body(builder: Builder, config: BlockConfig, x: Act, stream_sink=None, grad_sink=None) -> Act:
    """the block's layers (+ skip), run inside an already-entered block scope"""
    skip = config.skip and config.memory_reduction_strategy in ("none", "checkpoint")
    out, consumed = run_layers(builder, list(config.layer), x, residual=x if skip else None,
                               stream_sink=stream_sink, grad_sink=grad_sink)
    if skip and not consumed:
        out = Act(F.add(out.t, x.t), out.dims)
    return out


def block_scope_name(depth: int, config_idx: int, prefix: str = "") -> str:
    return f"{prefix}{depth}_{config_idx}"


def block_part_fn(builder: Builder, config: BlockConfig, x: Act, depth: int, config_idx: int,
                  prefix: str = "") -> Act:
    builder.depth_idx, builder.config_idx = depth, config_idx
    with builder.scope.exact(block_scope_name(depth, config_idx, prefix)):
        return block_body(builder, config, x)
