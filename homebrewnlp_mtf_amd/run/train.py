"""`train` run mode: the host step loop (ref src/run/run.py:217-262 hot loop, src/main.py:44-166 driver).

Per rank: build the trainer, resume from the newest complete checkpoint (variables, optimizer slots, step and the
exact data cursor), then run ``macro_batching`` optimizer steps per host iteration until ``train_steps``.
Every ``log_every`` steps rank 0 syncs once and writes loss / accuracy / learning rate / tokens/s / TFLOP/s
(JSONL + TensorBoard) and every rank touches its heartbeat file for the watchdog (tools/run_manager.py).
Fault injection for resume tests: ``FI_KILL_AT_STEP=N`` (optionally ``FI_KILL_RANK=r``) hard-exits after step N.
"""
from __future__ import annotations

import json
import os
import time
import typing

import torch

from ..config import ModelParameter
from ..data import pipeline as data
from ..models.model import count_flops_per_token
from ..parallel import launch
from ..utils import checkpoint as ckpt
from ..utils.log import log
from ..utils.metrics import MetricsWriter, analyze_model, grad_norms
from .trainer import Trainer

PEAK_BF16_DENSE = 2.5e15


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _mean_over_ranks(vals: dict, dev) -> dict:
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return vals
    keys = [k for k, v in vals.items() if isinstance(v, torch.Tensor) and v.numel() == 1]
    if not keys:
        return vals
    t = torch.stack([vals[k].detach().float().reshape(()).to(dev) for k in keys])
    dist.all_reduce(t)
    t /= dist.get_world_size()
    out = dict(vals)
    out.update({k: t[i] for i, k in enumerate(keys)})
    return out


def train(params: ModelParameter, debug_grad: bool = False, synthetic: bool = False, device: str = "auto",
          max_steps: typing.Optional[int] = None) -> dict:
    mesh, dev = launch.init(params, device)
    rank = mesh.rank
    model_path = params.model_path
    if rank == 0:
        os.makedirs(model_path, exist_ok=True)
        with open(os.path.join(model_path, f"run_config_{int(time.time())}.json"), "w") as f:
            json.dump(params.dict(), f, indent=2, default=str)
    trainer = Trainer(params, dev, mesh)
    if rank == 0:
        analyze_model(trainer.store, os.path.join(model_path, "model_size.info"))
    step, data_state = 0, None
    if params.use_checkpointing:
        path = ckpt.latest(model_path)
        if path:
            step, data_state = ckpt.restore(trainer, path)
            log(f"resumed from {path} at step {step}")
    trainer.global_step = step
    if params.model_mode == "jannet":
        from ..data import video
        if synthetic or not params.dataset_configs:
            feeder = video.SyntheticVideo(params, trainer.local_batch, dev, seed=1000 * mesh.dp_rank + step)
        else:
            feeder = video.jannet_input(params, trainer.local_batch, mesh.dp_rank, mesh.dp, dev)
            if data_state is not None and hasattr(feeder, "restore"):
                feeder.restore(data_state)
    elif synthetic or not params.dataset_configs:
        feeder = data.SyntheticText(params, trainer.local_batch, dev, seed=1000 * mesh.dp_rank + step)
    else:
        feeder = data.text_input(params, trainer.local_batch, mesh.dp_rank, mesh.dp, dev, state=data_state,
                                 prefetch=int(params.buffer_size or 4))
    metrics = MetricsWriter(params.metrics_path or os.path.join(model_path, "metrics.jsonl"),
                            os.path.join(model_path, "tensorboard") if params.tensorboard else None,
                            enabled=rank == 0)
    heartbeat = params.heartbeat_path or os.path.join(model_path, f"heartbeat-r{rank:04d}")
    fi_step = int(os.environ.get("FI_KILL_AT_STEP", "-1"))
    fi_rank = int(os.environ.get("FI_KILL_RANK", "0"))
    flops_tok = count_flops_per_token(params, trainer.store)
    tokens_per_step = params.train_batch_size * params.sequence_length
    end = params.train_steps if max_steps is None else min(params.train_steps, step + max_steps)
    log_every = max(1, int(params.log_every))
    last_log_t, last_log_step = time.time(), step
    out: typing.Dict[str, typing.Any] = {}
    last_saved = step
    while step < end:
        k = min(int(params.macro_batching), end - step)
        batches = []
        for _ in range(k):
            b = feeder.next()
            if b is None:
                break
            batches.append(b)
        if not batches:
            log("input data exhausted")
            break
        m = trainer.train_steps(batches)
        step += len(batches)
        if debug_grad:
            m.update(grad_norms(trainer.store))
        if step % log_every == 0 or step >= end:
            _sync(dev)
            now = time.time()
            tps = (step - last_log_step) * tokens_per_step / max(now - last_log_t, 1e-9)
            vals = _mean_over_ranks({k2: v for k2, v in m.items()}, dev)     # X07: losses averaged over ranks
            vals.update(tokens_per_s=tps, tflops_per_gpu=tps * flops_tok / mesh.world / 1e12,
                        mfu=tps * flops_tok / mesh.world / PEAK_BF16_DENSE if dev.type == "cuda" else 0.0)
            metrics.write(step, vals)
            out = {k2: (float(v) if isinstance(v, (int, float, torch.Tensor)) else v) for k2, v in vals.items()
                   if not k2.startswith("grad_norm/")}
            if rank == 0:
                log(f"step {step}: loss={out['loss']:.4f} acc={out.get('accuracy', 0.0):.4f} "
                    f"lr={out['learning_rate']:.3g} tokens/s={tps:.0f}")
            with open(heartbeat, "w") as f:
                f.write(f"{now} {step}\n")
            last_log_t, last_log_step = now, step
        if step == fi_step and rank == fi_rank:
            log(f"fault injection: killing rank {rank} after step {step}")
            os._exit(17)
        if params.use_checkpointing and step % int(params.steps_per_checkpoint) == 0:
            ckpt.save(trainer, model_path, step, feeder.consumed_state, keep=int(params.max_checkpoints_keep))
            last_saved = step
    if params.use_checkpointing and step != last_saved:
        ckpt.save(trainer, model_path, step, feeder.consumed_state, keep=int(params.max_checkpoints_keep))
    feeder.close()
    metrics.close()
    out["step"] = step
    return out
