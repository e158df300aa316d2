"""Named-dimension algebra that decides every weight shape of the block grammar.

Behavioural parity with the reference's ``linear_shapes`` / ``get_intermediate`` / ``get_attention_dim`` /
``get_fan_in`` (``src/utils_mtf.py:376-436``). Activations here are plain torch tensors plus a static tuple of
``Dim(name, size)`` describing their axes; the algebra runs once per call on those tuples (no graph, no lowering).
"""
from __future__ import annotations

import typing

from ..config import Dim, anonymize_dim

DimList = typing.List[Dim]
LinearShapes = typing.NamedTuple("LinearShapes", (("old", DimList), ("new", DimList)))
AttentionDim = typing.NamedTuple("AttentionDim", (("index", int), ("dim", Dim)))


def deduplicate(dims: typing.Iterable[Dim]) -> DimList:
    out = []
    for d in dims:
        if d not in out:
            out.append(d)
    return out


def subtract(a: typing.Iterable[Dim], b: typing.Iterable[Dim]) -> DimList:
    b = list(b)
    return [d for d in a if d not in b]


def crossection(*shapes: typing.Iterable[Dim]) -> DimList:
    shapes = [list(s) for s in shapes]
    alld = deduplicate(d for s in shapes for d in s)
    return [d for d in alld if all(d in s for s in shapes)]


def size(dims: typing.Iterable[Dim]) -> int:
    out = 1
    for d in dims:
        out *= d.size
    return out


def get_intermediate(params, extras) -> DimList:
    """ref ``src/utils_mtf.py:376-380``."""
    if 'group' not in extras:
        return list(params.intermediate)
    return [params.head_dim, anonymize_dim(params.key_dim, params.key_dim.size * params.group_linear_factor)]


def linear_shapes(params, extras, tensor_dims: DimList) -> LinearShapes:
    """ref ``src/utils_mtf.py:383-391``: which input dims a linear contracts (``old``) and which it creates (``new``).

    ``group`` keeps ``heads`` as a batch (block-diagonal) dimension."""
    features = get_intermediate(params, extras) + list(params.feature_dims)
    if 'group' in extras and params.intermediate[-1] in tensor_dims:
        features.remove(params.key_dim)
        features.extend(params.intermediate)
    features = deduplicate(features)
    old = crossection(tensor_dims, features)
    keep_head = [params.head_dim] if 'group' in extras and params.head_dim in old else []
    new = subtract(features, subtract(old, keep_head))
    return LinearShapes(old, new)


def feature_dims_used(params, dims: DimList) -> bool:
    """ref ``src/utils_mtf.py:360-367``."""
    fd = list(params.feature_dims) + [anonymize_dim(d) for d in params.feature_dims]
    return bool(sum(f in dims for f in fd) // 2)


def get_fan_in(params, dims: DimList) -> DimList:
    """ref ``src/utils_mtf.py:429-436``."""
    dims = list(dims)
    if feature_dims_used(params, dims) and params.key_dim in dims and dims.index(params.key_dim) == len(dims):
        return dims[:-2]  # unreachable in the reference as well (index == len); kept for parity
    if feature_dims_used(params, dims):
        return dims[:2]
    return dims[:1]


def get_attention_dim(params, tensor_dims: DimList) -> AttentionDim:
    """ref ``src/utils_mtf.py:418-422``: attention cycles over the non-feature spatial dims (batch excluded)."""
    dims = subtract(subtract(tensor_dims, params.feature_dims), params.intermediate)[1:]
    idx = params.attention_idx % len(dims)
    return AttentionDim(idx, dims[idx])


def is_masked(params, tensor_dims: DimList) -> bool:
    return get_attention_dim(params, tensor_dims).index in params.masked_attention_dimensions
