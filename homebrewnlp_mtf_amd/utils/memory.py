"""Per-rank HBM sizing of a training step (masters, gradients, optimizer slots, activations).

The static part is exact: the model's registration pass runs on meta tensors at the requested ``(tp_rank, tp)``
(``Model(..., finalize=False)``) and yields every variable's local shape; each local parameter then costs
  4 B fp32 master + 4 B fp32 gradient + 2 B bf16 compute copy + 2 B bf16 transposed copy (``ParamStore.transposed``)
plus the fused optimizer's fp32 buffers for the chain (``optim/fused.py``: momentum 4 B, Adam 8 B, NovoGrad /
Adafactor 4 B, two chain-output temporaries ``u``/``u2`` 4 B each, SM3 accumulators per dimension, double-buffered).

Activations follow the tensors the fused autograd ops save (``ops/functional.py``) for the reference's TP layout
(``src/dataclass.py:247-252``: the residual stream and every per-head tensor are sharded over the ``heads`` axis, the
``intermediate`` axis is replicated -- tp_layout "heads"), per token and layer, bf16 unless noted:
  norm          output 2 F/tp + fp32 row stats 8
  attention     in-projection output ("base") 2 I, k|q|v 6 F/tp, attention output 2 F/tp, fp32 lse 4 H/tp,
                block output (residual sum) 2 F/tp
  feed_forward  pre-activation 2 I (+ activation output 2 I with an activation), block output 2 F/tp
(tp_layout "intermediate" divides the I terms by tp as well). With GPT-Neo-1.3B at 64 x 2048 tokens on one GPU
this gives 182 GB of activations + 32 GB static = 214 GB against the 200 GiB (215 GB) measured peak
(bench.py, round 3); the estimate is 227 GB (conservative by 6 %). The GPU test
``test_gpt_neo_20b_tp8_fits_per_rank`` checks the 20B-scale TP8 shard against eight gloo ranks on one MI355X. Memory strategies: ``none`` keeps every layer; ``checkpoint`` keeps block inputs
and recomputes one block; ``revnet`` / ``momentum`` keep the two streams plus one block's worth (O(1) in depth).
"""
from __future__ import annotations

import typing

def _layer_bytes(layer: str, F: int, I: int, H: int, tp: int, itp: bool) -> float:
    """saved bytes per token of one layer string of a block (see module docstring)"""
    name = layer.split("-")[0]
    extras = layer.split("-")[1:]
    i_loc = I / tp if itp else I
    if name == "norm":
        return 2 * F / tp + 8
    if name == "attention":
        if "biased_attention_map" in extras or "input_as_value" in extras:   # token mixer: input + output
            return 2 * i_loc + 4 * F / tp
        return 2 * i_loc + 6 * F / tp + 2 * F / tp + 4 * H / tp + 2 * F / tp
    if name in ("feed_forward", "bottleneck_group_linear", "product_key_memory", "feed_forward_product_key_memory"):
        act = any(e.startswith("in:") and len(e) > 3 for e in extras) or name != "feed_forward"
        return 2 * i_loc * (2 if act else 1) + 2 * F / tp
    # group_linear, rezero, activation, dropout, cumsum, ...: input-sized
    return 4 * F / tp


def _optimizer_bytes_per_param(chain: str) -> float:
    stages = [s.split(":")[0] for s in str(chain).split("-")]
    b = 0.0
    if "momentum" in stages or "nesterov" in stages:
        b += 4
    if "adam" in stages:
        b += 8
    if "novograd" in stages or "adafactor" in stages:
        b += 4
    b += 8   # chain-output temporaries u, u2 (fp32), allocated when the chain has more than one output segment
    return b


def estimate(params, dp: int = 1, tp: int = 1, local_batch: typing.Optional[int] = None) -> typing.Dict[str, float]:
    """bytes per rank of one training step of ``params`` on a ``dp x tp`` mesh (rank 0 of its TP group)"""
    from ..models.model import Model, padded_vocab

    if local_batch is None:
        local_batch = max(int(params.train_batch_size) // max(dp, 1), 1)
    m = Model(params, "meta", tp_rank=0, tp_size=tp, local_batch=local_batch, finalize=False)
    specs = m.store.specs
    n_local = sum(s.numel for s in specs.values())
    sm3 = 0
    if "sm3" in str(params.optimizer):
        sm3 = sum(sum(int(d) for d in s.local_shape) for s in specs.values()) * 4 * 2
    param_bytes = n_local * (4 + 4 + 2 + 2)
    opt_bytes = n_local * _optimizer_bytes_per_param(params.optimizer) + sm3

    F = int(params.features)
    I = int(params.intermediate[0].size) if params.intermediate else 2 * F
    H = int(params.heads)
    itp = getattr(params, "tp_layout", "heads") == "intermediate"
    T = local_batch * int(params.sequence_length)
    per_layer = sum(_layer_bytes(layer, F, I, H, tp, itp) for bc in params.block_configs for layer in bc.layer)
    per_layer_bytes = T * per_layer
    strategy = str(params.memory_reduction_strategy)
    depth = int(params.depth)
    # none: every layer's saved tensors; checkpoint: one block recomputed at a time (its inputs: stream_bytes);
    # revnet / momentum: the two streams plus one block recomputed
    layers_kept = depth if strategy == "none" else 1
    stream_bytes = 0.0 if strategy == "none" else T * (2 * F / tp) * (depth if strategy == "checkpoint" else 4)
    V = padded_vocab(params)
    # logits (bf16; the cross-entropy backward writes their gradient in place), embedding output and its gradient,
    # the widest layer's backward transients (dz, dx)
    other = T * (2 * V + 4 * F / tp + 2 * (I / tp if itp else I) * 2) + stream_bytes
    act_bytes = layers_kept * per_layer_bytes + other
    total = param_bytes + opt_bytes + act_bytes
    del m
    return {"params_local": float(n_local), "param_bytes": float(param_bytes), "optimizer_bytes": float(opt_bytes),
            "activation_bytes_per_layer": float(per_layer_bytes), "activation_bytes_other": float(other),
            "activation_bytes": float(act_bytes), "total_bytes": float(total), "tokens_local": float(T)}
