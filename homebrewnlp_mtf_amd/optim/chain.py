"""Optimizer chain grammar and learning-rate schedule.

Chain: ``"name:arg:arg-name-..."`` (ref src/optimizer/__init__.py:42-44), e.g.
``"adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate"``. Stages: adam, sm3, novograd, adafactor (new; not in
the reference), momentum, adaptive_clip, l2norm_clip, global_l2norm_clip, value_clip, gradient_centralisation,
weight_centralisation, learning_rate, graft.

LR: ``learning_rate`` x each module of ``learning_rate_config`` in config order (ref
src/optimizer/learning_rate.py:27-72): linear_warmup, exponential_decay, linear_decay, lower_bound, upper_bound.
"""
from __future__ import annotations

import typing

KNOWN = ("adam", "sm3", "novograd", "adafactor", "momentum", "adaptive_clip", "l2norm_clip", "global_l2norm_clip",
         "value_clip", "gradient_centralisation", "weight_centralisation", "learning_rate", "graft")

Stage = typing.Tuple[str, typing.Tuple[str, ...]]


def parse_chain(chain: str) -> typing.List[Stage]:
    out = []
    for part in chain.split('-'):
        if not part:
            continue
        name, *args = part.split(':')
        if name not in KNOWN:
            raise ValueError(f"unknown optimizer stage {name!r}; known: {KNOWN}")
        out.append((name, tuple(args)))
    return out


def learning_rate(params, global_step: int) -> float:
    lr = float(params.learning_rate)
    step = float(global_step)
    for name, cfg in params.learning_rate_modules.items():
        if name == "linear_warmup":
            warm = float(cfg.final_step)
            lr *= step / warm if step < warm else 1.0
        elif name == "exponential_decay":
            lr *= float(cfg.factor) ** max(step - float(cfg.start_step), 0.0)
        elif name == "linear_decay":
            cur = step - float(cfg.start_step)
            fin = float(cfg.final_step) - float(cfg.start_step)
            lr *= min(max(1.0 - cur / fin, 0.0), 1.0)
        elif name == "lower_bound":
            lr = max(lr, float(cfg.factor))
        elif name == "upper_bound":
            lr = min(lr, float(cfg.factor))
        else:
            raise ValueError(f"unknown learning-rate module {name!r}")
    return lr
