"""Sharded checkpoints with reference-style names (ref src/run/run.py:158-175 Saver + CheckpointSaverHook,
src/run/utils_run.py:18-29 CheckpointLoaderHook, src/main.py:71 resume step).

Layout under ``model_path``::

    checkpoint                  latest complete checkpoint directory name (atomically replaced)
    ckpt-000001000/
      meta.json                 step, mesh, format, config, shard list
      tp00-of-02.bin / .json    fp32 tensors of TP rank 0: every variable (its TP shard) and every optimizer slot
      data-r0003.npy            exact loader cursor of global rank 3 (one per rank)

Names are the variable scope paths (``gpt0/body0/0_0/attention_0/linear0/orthogonal_var0``) and slots follow the
reference's ``<var>/<optimizer string with : -> _>/<slot>`` (src/optimizer/backend.py:23-25). Every tensor carries
its local shape, global shape and TP dimension, so a checkpoint restores into a different TP degree (variables and
the slots shaped like them are re-sliced; SM3 accumulators of the split dim are concatenated).
Writes go to ``ckpt-X.tmp`` (native parallel blob IO with per-piece CRC32C, fsync) and are renamed only when every
rank finished, then the oldest checkpoints beyond ``max_checkpoints_keep`` are removed.
"""
from __future__ import annotations

import json
import os
import shutil
import time
import typing

import numpy as np
import torch
import torch.distributed as dist

from . import blobio

FORMAT = "obst-ckpt-v1"


def _barrier():
    if dist.is_initialized():
        dist.barrier()


def _dirname(step: int) -> str:
    return f"ckpt-{step:09d}"


def latest(model_path: str) -> typing.Optional[str]:
    ptr = os.path.join(model_path, "checkpoint")
    if os.path.exists(ptr):
        name = open(ptr).read().strip()
        path = os.path.join(model_path, name)
        if os.path.exists(os.path.join(path, "meta.json")):
            return path
    # fall back to scanning (pointer lost)
    if not os.path.isdir(model_path):
        return None
    done = sorted(d for d in os.listdir(model_path) if d.startswith("ckpt-") and not d.endswith(".tmp")
                  and os.path.exists(os.path.join(model_path, d, "meta.json")))
    return os.path.join(model_path, done[-1]) if done else None


def latest_step(model_path: str) -> int:
    p = latest(model_path)
    if p is None:
        return 0
    return int(json.load(open(os.path.join(p, "meta.json")))["step"])


# ---------------------------------------------------------------------------------------------------------------
def _slot_tp_dim(slot_key: str, var_tp: typing.Optional[int], slot_shape, var_shape) -> typing.Tuple[
        typing.Optional[int], bool]:
    """(tp dim of a slot, whether it can be re-sliced)"""
    if var_tp is None:
        return None, True
    leaf = slot_key.rsplit("/", 1)[-1]
    if list(slot_shape) == list(var_shape):
        return var_tp, True
    if leaf.startswith("dim"):
        return (0 if int(leaf[3:]) == var_tp else None), True
    if leaf in ("af_rows", "af_cols"):
        # Adafactor factors of [rows = leading dims flattened, cols = last dim] (optim/reference.py _adafactor):
        # the factor over the sharded axis is local, the other one is the TP-reduced (replicated) statistic
        last = len(var_shape) - 1
        if leaf == "af_cols":
            return (0 if var_tp == last else None), True
        # af_rows: replicated when the last dim is sharded; else sharded along var_tp of the rows' unflattened view
        # [leading dims] (a sharded middle dim interleaves the local rows: re-sliced through that view, _TP_VIEW)
        return (None, True) if var_tp == last else (var_tp, True)
    return None, True      # scalars (TP-summed statistics) are replicated


def _tp_view(slot_key: str, var_tp, var_shape):
    """the unflattened local shape a flattened sharded slot is re-sliced in (Adafactor row factors), or None"""
    if var_tp is not None and slot_key.rsplit("/", 1)[-1] == "af_rows" and var_tp != len(var_shape) - 1:
        return [int(d) for d in var_shape[:-1]]
    return None


def _named_tensors(trainer) -> typing.Dict[str, typing.Tuple[torch.Tensor, dict]]:
    store = trainer.store
    out = {}
    tp = trainer.mesh.tp
    for name in store.order:
        s = store.specs[name]
        local = list(s.local_shape)
        glob = [d.size for d in s.dims]
        out[name] = (store.master_view(name), {"kind": "variable", "shape": local, "global_shape": glob,
                                                "tp_dim": s.tp_dim, "resliceable": True})
    slots = trainer.opt.named_slots()
    for key, t in slots.items():
        var = key.split("/" + trainer.params.optimizer.replace(":", "_") + "/", 1)[0]
        s = store.specs[var]
        tp_dim, ok = _slot_tp_dim(key, s.tp_dim, t.shape, s.local_shape)
        view = _tp_view(key, s.tp_dim, s.local_shape)
        glob = list(t.shape)
        if view is not None:
            glob = [int(t.numel()) * tp]
        elif tp_dim is not None:
            glob[tp_dim] *= tp
        meta = {"kind": "slot", "shape": list(t.shape), "global_shape": glob, "tp_dim": tp_dim, "resliceable": ok}
        if view is not None:
            meta["tp_view"] = view
        out[key] = (t, meta)
    return out


def save(trainer, model_path: str, step: int, data_state: typing.Optional[np.ndarray] = None,
         keep: int = 1, extra: typing.Optional[dict] = None) -> str:
    mesh = trainer.mesh
    rank = mesh.rank
    final = os.path.join(model_path, _dirname(step))
    tmp = final + ".tmp"
    if rank == 0:
        os.makedirs(model_path, exist_ok=True)
        if os.path.exists(tmp):
            shutil.rmtree(tmp)
        os.makedirs(tmp)
    _barrier()
    t0 = time.time()
    if mesh.dp_rank == 0:   # one writer per TP shard
        named = _named_tensors(trainer)
        total = sum(t.numel() for t, _ in named.values())
        pin = trainer.device.type == "cuda"
        arena = torch.empty(total, dtype=torch.float32, pin_memory=pin)
        views, off = [], 0
        for name, (t, _) in named.items():
            v = arena[off:off + t.numel()]
            v.copy_(t.detach().reshape(-1).float(), non_blocking=pin)
            views.append(v)
            off += t.numel()
        if pin:
            torch.cuda.synchronize(trainer.device)
        base = f"tp{mesh.tp_rank:02d}-of-{mesh.tp:02d}"
        meta = blobio.write_blobs(os.path.join(tmp, base + ".bin"), views)
        crcs = blobio.piece_crcs(meta)
        index = {}
        for i, (name, (_, info)) in enumerate(named.items()):
            index[name] = dict(info, dtype="float32", offset=meta["offsets"][i], nbytes=meta["sizes"][i],
                               crcs=crcs[i])
        with open(os.path.join(tmp, base + ".json"), "w") as f:
            json.dump({"format": FORMAT, "tp_rank": mesh.tp_rank, "tp": mesh.tp, "tensors": index}, f)
    if data_state is not None:
        np.save(os.path.join(tmp, f"data-r{rank:04d}.npy"), np.asarray(data_state, dtype=np.int64))
    _barrier()
    if rank == 0:
        meta = {"format": FORMAT, "step": int(step), "dp": mesh.dp, "tp": mesh.tp, "world": mesh.world,
                "optimizer": trainer.params.optimizer, "time": time.time(), "write_seconds": time.time() - t0,
                "shards": [f"tp{r:02d}-of-{mesh.tp:02d}" for r in range(mesh.tp)]}
        if extra:
            meta.update(extra)
        with open(os.path.join(tmp, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.rename(tmp, final)
        ptr = os.path.join(model_path, "checkpoint")
        with open(ptr + ".tmp", "w") as f:
            f.write(os.path.basename(final) + "\n")
        os.replace(ptr + ".tmp", ptr)
        done = sorted(d for d in os.listdir(model_path) if d.startswith("ckpt-") and not d.endswith(".tmp"))
        for d in done[:max(0, len(done) - max(1, keep))]:
            shutil.rmtree(os.path.join(model_path, d), ignore_errors=True)
    _barrier()
    return final


# ---------------------------------------------------------------------------------------------------------------
class _ShardReader:
    def __init__(self, path: str, base: str):
        self.bin = os.path.join(path, base + ".bin")
        self.index = json.load(open(os.path.join(path, base + ".json")))["tensors"]

    def read(self, names: typing.List[str]) -> typing.Dict[str, torch.Tensor]:
        bufs = [torch.empty(self.index[n]["nbytes"] // 4, dtype=torch.float32) for n in names]
        meta = {"offsets": [self.index[n]["offset"] for n in names], "sizes": [self.index[n]["nbytes"] for n in names],
                "crcs": [c for n in names for c in self.index[n]["crcs"]]}
        blobio.read_blobs(self.bin, bufs, meta)
        return {n: b.view(self.index[n]["shape"]) for n, b in zip(names, bufs)}


def restore(trainer, path: str, strict: bool = True) -> typing.Tuple[int, typing.Optional[np.ndarray]]:
    """Loads variables + optimizer slots into the trainer; returns (step, this rank's data cursor or None)."""
    meta = json.load(open(os.path.join(path, "meta.json")))
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: unknown checkpoint format {meta.get('format')}")
    mesh = trainer.mesh
    old_tp = int(meta["tp"])
    readers = [_ShardReader(path, b) for b in meta["shards"]]
    named = _named_tensors(trainer)
    index0 = readers[0].index
    opt_tag = "/" + trainer.params.optimizer.replace(":", "_") + "/"
    missing = [n for n in named if n not in index0]
    if missing and strict:
        raise KeyError(f"checkpoint lacks {len(missing)} tensors, e.g. {missing[:3]}")
    # slots the (lazy) reference optimizer has not created yet are loaded too
    wanted = [n for n in named if n in index0] + [n for n, i in index0.items() if i["kind"] == "slot"
                                                   and n not in named and opt_tag in n]
    if old_tp == mesh.tp:
        loaded = readers[mesh.tp_rank].read(wanted)
    else:
        loaded = {}
        sharded = [n for n in wanted if index0[n]["tp_dim"] is not None]
        repl = [n for n in wanted if index0[n]["tp_dim"] is None]
        loaded.update(readers[0].read(repl))
        parts = [r.read(sharded) for r in readers]
        for n in sharded:
            info = index0[n]
            if not info["resliceable"]:
                raise ValueError(f"{n} cannot be re-sliced from TP={old_tp} to TP={mesh.tp}")
            view = info.get("tp_view")
            full = torch.cat([p[n].view(view) if view else p[n] for p in parts], info["tp_dim"])
            k = full.shape[info["tp_dim"]] // mesh.tp
            loaded[n] = full.narrow(info["tp_dim"], mesh.tp_rank * k, k).contiguous()
            if view:
                loaded[n] = loaded[n].reshape(-1)
    lazy = {}
    with torch.no_grad():
        for n in wanted:
            src = loaded[n]
            if n not in named:
                lazy[n] = src
                continue
            dst, _ = named[n]
            if list(src.shape) != list(dst.shape):
                raise ValueError(f"{n}: checkpoint shape {list(src.shape)} vs model {list(dst.shape)}")
            dst.copy_(src.to(dst.device))
    if lazy:
        from ..optim.reference import ReferenceOptimizer
        if not isinstance(trainer.opt, ReferenceOptimizer):
            raise KeyError(f"optimizer has no slot {next(iter(lazy))}")
        trainer.opt.load_state_dict(lazy)
    trainer.store.sync_compute()
    data = os.path.join(path, f"data-r{mesh.rank:04d}.npy")
    state = np.load(data) if os.path.exists(data) and int(meta["world"]) == mesh.world else None
    trainer.global_step = int(meta["step"])
    return int(meta["step"]), state
