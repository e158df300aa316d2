"""Training runtime: model + optimizer + DP gradient sync + step loop (ref src/run/run.py:27-262, train.py:19-77).

One process per GPU. ``Trainer.step(batches)`` runs one optimizer step over ``grad_accumulation`` micro-batches
(gradient accumulation, bug A11 fixed): forward, backward (weight gradients land in the flat fp32 buffer, DP
buckets all-reduce while backward runs), then the fused optimizer. ``macro_batching`` (K optimizer steps per host
call, ref train.py:21-74) is ``train_steps``. Metrics stay on device; the host syncs only when it logs.
"""
from __future__ import annotations

import os
import time
import typing

import torch
import torch.distributed as dist

from ..config import ModelParameter
from ..models.model import Model
from ..optim import fused as fused_opt
from ..optim.chain import learning_rate
from ..optim.reference import ReferenceOptimizer
from ..parallel import state as pstate
from ..parallel.grad_sync import GradSync
from ..utils import debug
from ..utils.log import log


class Trainer:
    def __init__(self, params: ModelParameter, device: typing.Union[str, torch.device] = "cpu",
                 mesh: typing.Optional[pstate.Mesh] = None, dtype: typing.Optional[torch.dtype] = None,
                 use_fused: typing.Optional[bool] = None):
        self.params = params
        self.device = torch.device(device)
        self.mesh = mesh or pstate.mesh()
        pstate.set_mesh(self.mesh)
        if params.train_batch_size % self.mesh.dp:
            raise ValueError("train_batch_size must be divisible by dp")
        self.local_batch = params.train_batch_size // self.mesh.dp
        t0 = time.time()
        self.model = Model(params, self.device, self.mesh.tp_rank, self.mesh.tp, dtype=dtype,
                           local_batch=self.local_batch)
        self.store = self.model.store
        log(f"model built in {time.time() - t0:.1f}s: {self.store.global_numel() / 1e6:.2f}M parameters "
            f"({len(self.store.specs)} tensors), local {self.store.numel() / 1e6:.2f}M")
        if use_fused is None:
            use_fused = self.device.type == "cuda" and fused_opt.supported(params.optimizer)
            if self.device.type == "cuda" and not use_fused:
                log(f"WARNING: optimizer chain {params.optimizer!r} has no fused HIP plan "
                    f"({fused_opt.unsupported_reason(params.optimizer)}): the whole step falls back to the "
                    f"per-tensor torch ReferenceOptimizer on the GPU")
        self.opt = fused_opt.FusedOptimizer(self.store, params) if use_fused else ReferenceOptimizer(self.store,
                                                                                                        params)
        self.grad_sync = GradSync(self.store, self.mesh.dp_group, self.mesh.dp, params.grad_bucket_mb,
                                  {"float32": torch.float32, "bfloat16": torch.bfloat16}[params.allreduce_dtype],
                                  use_counts=self.model.builder.use_counts,
                                  force=bool(getattr(params, "force_grad_sync", False)))
        self.global_step = int(params.current_step)

    # ---------------------------------------------------------------------------------------------------------------
    def _micro_batches(self, batch: typing.Dict[str, torch.Tensor]) -> typing.List[typing.Dict[str, torch.Tensor]]:
        n = int(self.params.grad_accumulation)
        if n == 1:
            return [batch]
        out = []
        for i in range(n):
            out.append({k: (None if v is None else v.chunk(n, 0)[i]) for k, v in batch.items()})
        return out

    def step(self, batch: typing.Dict[str, torch.Tensor]) -> typing.Dict[str, torch.Tensor]:
        """one optimizer step; returns device-side metrics"""
        p = self.params
        if p.multi_loss_strategy in ("pcgrad", "mgda") and p.use_video and p.use_language:
            return self._multi_loss_step(batch)
        if p.use_hip_graphs and self._graphs_ok():
            return self._graph_step(batch)
        lr = learning_rate(self.params, self.global_step)
        metrics = self._step_body(batch, lr)
        self.global_step += 1
        metrics["learning_rate"] = torch.tensor(lr)
        if debug.CHECK:
            debug.verify()
        return metrics

    def _step_body(self, batch: typing.Dict[str, torch.Tensor], lr: float) -> typing.Dict[str, torch.Tensor]:
        """zero grads, forward + backward over the micro-batches, DP sync, optimizer -- all device work of a step"""
        self.store.zero_grad()
        micro = self._micro_batches(batch)
        metrics: typing.Dict[str, torch.Tensor] = {}
        for i, mb in enumerate(micro):
            last = i == len(micro) - 1
            if last:
                self.grad_sync.attach()
            try:
                out = self.model(**mb, train=True, step_seed=self.global_step * 131 + i)
                loss = out["loss"] / len(micro)
                loss.backward()
            finally:
                self.grad_sync.detach()
            self.store.fold_leaf_grads()
            for k, v in out.items():
                v = v.detach().float()
                metrics[k] = metrics.get(k, 0) + v / len(micro)
        with debug.range_("dp_sync"):
            # the 1/dp mean is folded into the optimizer's gradient scale (no extra pass over the gradient buffer)
            self.grad_sync.finish(average=False)
        with debug.range_("optimizer"):
            self.opt.step(lr, self.global_step + 1, grad_scale=1.0 / max(self.mesh.dp, 1))
        return metrics

    # ---------------------------------------------------------------------------------------------------------------
    # Whole-step hipGraph (``use_hip_graphs``): the device work of a training step -- forward, backward (every HIP
    # kernel, gemm4w GEMM and allocation of the step), the fused optimizer -- is captured once and replayed, so
    # the host issues one graph launch per step instead of ~1000 kernel launches. The values that change between
    # steps live on the device (input tokens copied into static buffers, [lr, step] read by the optimizer kernels);
    # the SM3 accumulators alternate between two buffers, so one graph is captured per parity.
    def _graphs_ok(self) -> bool:
        p = self.params
        dropout = p.input_dropout > 0 or "dropout" in str(p.block_config)
        # world > 1: RCCL collectives can be captured (async all-reduce + wait become graph nodes), but only on the
        # nccl backend and only as an opt-in (hip_graphs_distributed): gloo runs on the host and cannot be captured.
        # The bf16 DP wire's all_to_all crashes inside hipStreamEndCapture on this image (round 6 probe:
        # profiles/r6_rccl_capture.md), so a captured multi-rank step needs the fp32 all-reduce wire
        multi_ok = self.mesh.world == 1 or (bool(getattr(p, "hip_graphs_distributed", False)) and dist.is_initialized()
                                            and dist.get_backend() == "nccl"
                                            and (self.mesh.dp == 1 or p.allreduce_dtype == "float32"))
        return (self.device.type == "cuda" and isinstance(self.opt, fused_opt.FusedOptimizer)
                and multi_ok and int(p.grad_accumulation) == 1 and not dropout
                and not getattr(self.store, "leaf_grads_seen", False) and not debug.CHECK)

    def _graph_step(self, batch: typing.Dict[str, torch.Tensor]) -> typing.Dict[str, torch.Tensor]:
        g = getattr(self, "_graph", None)
        if g is None:
            g = self._graph = {"inputs": {k: v.clone() for k, v in batch.items() if v is not None},
                               "graphs": {}, "warm": 0, "pool": torch.cuda.graph_pool_handle()}
            self.opt.external_dyn = True
        for k, v in batch.items():
            if v is not None:
                g["inputs"][k].copy_(v, non_blocking=True)
        lr = learning_rate(self.params, self.global_step)
        self.opt.set_dyn(lr, self.global_step + 1)
        parity = self.opt.flip
        if parity not in g["graphs"]:
            if g["warm"] < 2:     # eager warm-up: first-use GEMM plans, workspaces, allocator growth
                g["warm"] += 1
                metrics = self._step_body(g["inputs"], lr)
                self.global_step += 1
                metrics["learning_rate"] = torch.tensor(lr)
                return metrics
            self._capture(parity, lr)
        graph, out = g["graphs"][parity]
        graph.replay()
        self.opt.flip = 1 - parity
        self.store.bump()
        self.global_step += 1
        metrics = {k: v.clone() for k, v in out.items()}
        metrics["learning_rate"] = torch.tensor(lr)
        return metrics

    def _capture(self, parity: int, lr: float):
        """record the step for SM3 buffer parity ``parity`` (capture executes nothing on the device)"""
        g = self._graph
        keep = self.opt.flip
        self.opt.flip = parity
        graph = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        if dist.is_initialized() and dist.get_backend() == "nccl":
            # ProcessGroupNCCL's watchdog polls the events of finished eager collectives from its own thread (~every
            # 100 ms); a poll inside the capture aborts the process (profiles/r6_rccl_capture.md): let it reap them
            time.sleep(0.5)
        before = debug.comm_bytes()
        # OBST_CAPTURE_MODE (global | thread_local | relaxed): what other host threads may do while this one captures.
        # Multi-rank captures default to thread_local: ProcessGroupNCCL's watchdog polls its events from its own
        # thread, which a global-mode capture turns into an error (tools/graph_capture_probe.py)
        mode = os.environ.get("OBST_CAPTURE_MODE", "thread_local" if self.mesh.world > 1 else "global")
        with torch.cuda.graph(graph, pool=g["pool"], capture_error_mode=mode):
            out = self._step_body(g["inputs"], lr)
        # collectives recorded while capturing = what every replay issues (replays run no host code to count them)
        after = debug.comm_bytes()
        self.graph_comm = {k: (c - before.get(k, (0, 0))[0], b - before.get(k, (0, 0))[1])
                           for k, (c, b) in after.items() if c != before.get(k, (0, 0))[0]}
        self.opt.flip = keep     # capture ran the host side of the step (buffer flip) but executed nothing
        g["graphs"][parity] = (graph, out)
        log(f"captured the training step in a hipGraph (SM3 parity {parity})")

    def prepare_graphs(self) -> bool:
        """capture every parity's graph that the eager warm-up has not produced yet, so timed steps are replays
        only (benchmarks call this after their warm-up steps). False if graphs are not in use or not warm yet."""
        g = getattr(self, "_graph", None)
        if not (self.params.use_hip_graphs and self._graphs_ok()) or g is None or g["warm"] < 2:
            return False
        for parity in (0, 1):
            if parity not in g["graphs"]:
                self._capture(parity, learning_rate(self.params, self.global_step))
        return True

    def close(self) -> None:
        """release the captured step graphs (and their private memory pool) and the ops' cached scratch buffers"""
        from ..ops import functional as F
        self._graph = None
        F.release_workspaces()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()

    # ---------------------------------------------------------------------------------------------------------------
    def _multi_loss_step(self, batch):
        """token and video losses get separate (DP-averaged) gradients, combined per SURVEY A8 -- the reference
        wires pcgrad/mgda but never calls them (src/optimizer/gradients.py:65-66, __init__.py:102-126):
          pcgrad: g_i <- g_i - min(g_i . g_j, 0) / |g_j|^2 g_j per body variable (Yu et al. 2020), then summed;
          mgda:   two-task min-norm weight gamma from the body-gradient dot products (Sener & Koltun 2018; the
                  reference's min_gamma clamps), g = gamma g_token + (1 - gamma) g_video for every variable."""
        store = self.store
        micro = self._micro_batches(batch)
        parts = []
        metrics: typing.Dict[str, torch.Tensor] = {}
        for li, key in enumerate(("token_loss", "video_loss_raw")):
            store.zero_grad()
            for i, mb in enumerate(micro):
                out = self.model(**mb, train=True, step_seed=self.global_step * 131 + i)
                (out[key] / len(micro)).backward()
                store.fold_leaf_grads()
                if li == 0:
                    for k, v in out.items():
                        metrics[k] = metrics.get(k, 0) + v.detach().float() / len(micro)
            self.grad_sync.finish(average=True)
            parts.append(store.grad.clone())
        g1, g2 = parts
        body = [n for n in store.order if "body" in n]

        def dots(a, b):
            out = torch.stack([(store.grad_view_of(a, n) * store.grad_view_of(b, n)).sum() for n in body]) \
                if body else torch.zeros(0, device=a.device)
            sharded = torch.tensor([store.specs[n].tp_dim is not None for n in body], device=a.device)
            if pstate.tp_size() > 1 and body:
                part = out * sharded
                pstate.tp_all_reduce(part)
                out = torch.where(sharded, part, out)
            return out
        if self.params.multi_loss_strategy == "pcgrad":
            d12, d11, d22 = dots(g1, g2), dots(g1, g1), dots(g2, g2)
            out = g1 + g2
            for k, n in enumerate(body):
                c = torch.clamp(d12[k], max=0.0)
                v = store.grad_view_of(out, n)
                v.sub_(c / (d22[k] + 1e-20) * store.grad_view_of(g2, n) + c / (d11[k] + 1e-20) * store.grad_view_of(g1, n))
            store.grad.copy_(out)
        else:
            v11, v12, v22 = dots(g1, g1).sum(), dots(g1, g2).sum(), dots(g2, g2).sum()
            min_gamma = 0.001
            if float(v12) >= float(v11):
                gamma = 1 - min_gamma
            elif float(v12) >= float(v22):
                gamma = min_gamma
            else:
                gamma = float((v22 - v12) / (v11 + v22 - 2 * v12))
            store.grad.copy_(gamma * g1 + (1 - gamma) * g2)
            metrics["mgda_gamma"] = torch.tensor(gamma)
        lr = learning_rate(self.params, self.global_step)
        self.opt.step(lr, self.global_step + 1)
        self.global_step += 1
        metrics["learning_rate"] = torch.tensor(lr)
        return metrics

    def train_steps(self, batches: typing.Iterable[typing.Dict[str, torch.Tensor]]):
        """macro-batching: several optimizer steps per host call (first/last/mean loss, ref run.py:123-132)"""
        losses = []
        last = None
        for b in batches:
            last = self.step(b)
            losses.append(last["loss"])
        if not losses:
            return {}
        st = torch.stack(losses)
        out = dict(last)
        out.update(first_loss=st[0], last_loss=st[-1], mean_loss=st.mean())
        return out

    # ---------------------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def evaluate(self, batch) -> typing.Dict[str, torch.Tensor]:
        out = self.model(**batch, train=False)
        return {k: v.float() for k, v in out.items()}
