#!/usr/bin/env python3
"""Headline benchmark: training tokens/sec for the whole node, GPT-Neo-1.3B-shaped model, seq 2048, bf16
(BASELINE.json metric), one process per GPU over RCCL.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config configs/gpt_neo_1.3b.json] [--batch-per-gpu B]
                    [--tp T]

N > 1 is launched by the driver with ``torch.distributed.run`` (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in the env). A bare
``python bench.py --gpus N`` (no WORLD_SIZE) starts ``torch.distributed.run`` itself as a CHILD process, before anything
touches the GPU, and exits with its status (as ``main.py --gpus N`` does).
Weak scaling: every DP replica processes ``batch-per-gpu`` sequences per step (global batch = B x N / T). ``--tp T``
builds the reference's 2-D mesh (``src/dataclass.py:247-252``): ``Mesh(dp=N/T, tp=T)``, heads sharded over T
contiguous ranks -- BASELINE's GPT-Neo-2.7B at DP4 x TP2 and the 20B-scale config at TP8.
Each timed step is a full training step: forward, backward, DP all-reduce, fused optimizer update. Data is synthetic
(uniform random tokens, resident on the device) and the weights are randomly initialised.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from homebrewnlp_mtf_amd.config import load_config  # noqa: E402
from homebrewnlp_mtf_amd.models.model import count_flops_per_token  # noqa: E402
from homebrewnlp_mtf_amd.parallel import state as pstate  # noqa: E402
from homebrewnlp_mtf_amd.run.trainer import Trainer  # noqa: E402
from homebrewnlp_mtf_amd.utils.log import log  # noqa: E402

PEAK_BF16_DENSE = 2.5e15  # MI355X dense bf16 MFMA peak (spec, no sparsity)
TORCH_EAGER_1GPU = 80262.0  # tools/torch_baseline.py --batch 32 on one MI355X (profiles/r2_torch_baseline.md)


def _self_launch(n: int) -> int:
    """one process per GPU: ``torch.distributed.run`` as a child (never an exec: nothing here has touched the GPU)"""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults as the driver's command (--steps 20 --warmup 5): with 3 warm-up steps (the eager first step and the two
    # captures) the timed window starts on the first graph replays, which run slower -- 140.2k vs 150.6k tokens/s at
    # 10 / 3 vs 20 / 5 on one box (profiles/r6s/bench_defaults_ab.txt)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs",
                                                     "gpt_neo_1.3b.json"))
    # 64 sequences x 2048 tokens per GPU (200 GiB peak of the 288 GiB HBM3E): the optimizer step and the DP all-reduce
    # are per-step costs, so bigger per-GPU shards amortise them (one MI355X: 16 -> 32 -> 48 -> 64 sequences gave
    # 113.5k -> 121.4k -> 122.9k -> 123.6k tokens/s)
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="sequences per DP replica (default: 64 for GPT-Neo-1.3B, else the config's train_batch_size)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (heads sharded over T ranks)")
    ap.add_argument("--depth", type=int, default=0, help="(debug only: invalidates the headline number)")
    # the whole training step replayed as one hipGraph on a single GPU (1077 -> 1058 ms/step: the ~1500 launches of
    # a step no longer leave host-side gaps); with N > 1 ranks the step stays eager (RCCL all-reduces overlap it)
    # unless --hip-graphs-dist 1 (then with the fp32 all-reduce wire, the one the capture probe replays exactly)
    ap.add_argument("--hip-graphs", type=int, default=1, help="1: replay the captured training step (1 GPU)")
    ap.add_argument("--hip-graphs-dist", type=int, default=0,
                    help="1: capture the step with N > 1 ranks too (RCCL collectives inside the graph; opt-in)")
    ap.add_argument("--set", nargs="*", default=[], help="config overrides key=json_value (e.g. "
                    "revnet_stream_dtype=\"calculation\")")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: rehearse the launcher and the N-rank step on gloo (no GPU; not a measurement)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} != --gpus {args.gpus}")
    cpu = args.device == "cpu"
    # OBST_DIST_BACKEND=gloo rehearses the N-rank code path with several ranks sharing the visible GPUs (RCCL needs
    # one GPU per rank); the measured numbers always use the default, RCCL ("nccl") with one process per GPU
    backend = "gloo" if cpu else os.environ.get("OBST_DIST_BACKEND", "nccl")
    if cpu:
        args.hip_graphs = 0
        local_dev = 0
        device = torch.device("cpu")
    else:
        local_dev = local_rank % max(torch.cuda.device_count(), 1) if backend != "nccl" else local_rank
        torch.cuda.set_device(local_dev)
        device = torch.device("cuda", local_dev)

    def sync():
        if not cpu:
            torch.cuda.synchronize()
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
    tp = max(int(args.tp), 1)
    if world % tp:
        raise SystemExit(f"--tp {tp} does not divide the {world} ranks")
    dp = world // tp
    mesh = pstate.Mesh(dp=dp, tp=tp, rank=rank).build_groups()

    overrides = {}
    if not os.path.exists(args.config):   # relative to the repository (profilers run from elsewhere)
        args.config = os.path.join(os.path.dirname(os.path.abspath(__file__)), args.config)
    base = load_config(args.config)
    model_name = os.path.basename(args.config).replace(".json", "")
    if args.batch_per_gpu is None:
        args.batch_per_gpu = 64 if model_name == "gpt_neo_1.3b" else 0
    per_gpu = args.batch_per_gpu or base.train_batch_size
    if base.heads % tp:
        raise SystemExit(f"--tp {tp} does not divide the config's {base.heads} heads")
    overrides["train_batch_size"] = per_gpu * dp
    overrides["mesh"] = {"dp": dp, "tp": tp}
    if args.depth:
        overrides["depth"] = args.depth
    for item in args.set:
        k, _, v = item.partition("=")
        try:
            overrides[k] = json.loads(v)
        except json.JSONDecodeError:
            overrides[k] = v
    if args.hip_graphs:
        overrides["use_hip_graphs"] = True
        overrides["hip_graphs_distributed"] = bool(args.hip_graphs_dist)
        if args.hip_graphs_dist and dp > 1:
            # the capturable DP wire: one fp32 all-reduce per bucket (the bf16 wire's all_to_all does not survive
            # capture on this image, profiles/r6_rccl_capture.md)
            overrides["allreduce_dtype"] = "float32"
    params = load_config(args.config, overrides)
    torch.manual_seed(1234 + rank)
    trainer = Trainer(params, device, mesh)

    S = params.sequence_length
    B = trainer.local_batch
    gen = torch.Generator(device=device)
    gen.manual_seed(4321 + rank)
    batches = []
    for _ in range(4):
        toks = torch.randint(0, params.vocab_size, (B, S + 1, 1), device=device, generator=gen)
        batches.append({"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()})

    def barrier():
        if world > 1:
            if backend == "nccl":
                dist.barrier(device_ids=[local_dev])
            else:
                dist.barrier()

    t_w = time.time()
    from homebrewnlp_mtf_amd.utils import debug as obst_debug
    for i in range(args.warmup):
        m = trainer.step(batches[i % len(batches)])
        if i == 0:
            sync()
            log(f"first step done ({time.time() - t_w:.1f}s) loss={float(m['loss']):.4f} "
                f"peak mem {(0 if cpu else torch.cuda.max_memory_allocated(device)) / 2**30:.1f} GiB")
    trainer.prepare_graphs()    # record (not run) any step graph the warm-up has not captured: timed steps replay
    barrier()
    sync()
    obst_debug.comm_reset()
    t0 = time.perf_counter()
    for i in range(args.steps):
        m = trainer.step(batches[i % len(batches)])
    sync()
    barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed)
    peak = torch.tensor([0.0 if cpu else torch.cuda.max_memory_allocated(device) / 2 ** 30], dtype=torch.float64,
                        device=device)
    if world > 1:
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    peak = float(peak)
    comm = obst_debug.comm_bytes()   # collectives issued by this rank's timed steps (host count, replays excluded)
    graphs = bool(params.use_hip_graphs and trainer._graphs_ok())
    if graphs and world > 1:         # replays run no host code: per-step counts recorded at capture time
        comm = {k: [c * args.steps, b * args.steps] for k, (c, b) in getattr(trainer, "graph_comm", {}).items()}
    ms = 1000.0 * elapsed / max(args.steps, 1)
    tokens = params.train_batch_size * S * args.steps
    tps = tokens / elapsed
    fpt = count_flops_per_token(params, trainer.store)
    mfu = tps * fpt / (PEAK_BF16_DENSE * world)
    if rank == 0:
        log(f"loss={float(m['loss']):.4f} acc={float(m['accuracy']):.4f} step={ms:.1f}ms "
            f"tokens/s={tps:.0f} MFU={mfu * 100:.1f}% ({fpt / 1e9:.2f} GFLOP/token)")
        model = model_name
        metric = ("tokens/sec (whole node), GPT-Neo-1.3B seq2048 bf16" if model == "gpt_neo_1.3b" else
                  f"tokens/sec (whole node), {model} seq{S} bf16")
        from homebrewnlp_mtf_amd.ops import raw as obst_raw
        gemm = obst_raw.gemm_backend()
        if world > 1:
            per_step = {k: [c / max(args.steps, 1), round(b / max(args.steps, 1) / 2 ** 20, 2)]
                        for k, (c, b) in comm.items()}
            log(f"collectives per step on rank 0 ([calls, MiB]): {per_step}")
        print(json.dumps({
            "metric": metric,
            "value": round(tps, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (uniform random tokens), random-init weights",
            "mfu": round(mfu, 4), "final_loss": round(float(m["loss"]), 4),
            "peak_mem_gib": round(peak, 2),   # max over ranks of the allocator's peak (288 GB HBM3E per GPU)
            # informational: the plain PyTorch-ROCm eager run of the same model on one MI355X (80,262 tokens/s at
            # batch 32; profiles/r2_torch_baseline.md) -- BASELINE.md publishes no number, so vs_baseline stays null
            "vs_torch_eager_per_gpu": (round(tps / world / TORCH_EAGER_1GPU, 3) if model == "gpt_neo_1.3b" else None),
            "config": {"model": os.path.basename(args.config).replace(".json", "") +
                                (f"-depth{args.depth}(debug)" if args.depth else ""),
                       "global_batch": params.train_batch_size, "seq_len": S,
                       "set": args.set or None,
                       "revnet_stream": (params.revnet_stream_dtype if params.memory_reduction_strategy == "revnet"
                                         else None),
                       "parallelism": f"dp{dp}" + (f"xtp{tp}" if tp > 1 else ""),
                       "params": trainer.store.global_numel(), "optimizer": params.optimizer,
                       "hip_graphs": graphs,
                       # plain GEMMs: "gemm4w" = every product on the hand-written gfx950 kernel (no library GEMM)
                       "gemm": gemm,
                       "comm_mib_per_step": ({k: round(b / max(args.steps, 1) / 2 ** 20, 2)
                                              for k, (c, b) in comm.items()} if world > 1 else None),
                       # DP gradient reduction: buckets per step and wire dtype (bf16 = fp32-accumulated slices)
                       "dp_buckets": len(trainer.grad_sync.buckets) if dp > 1 else None,
                       "dp_wire": params.allreduce_dtype if dp > 1 else None,
                       "dp_wire_mib_per_step": (round(trainer.grad_sync.wire_bytes_per_step() / 2 ** 20, 1)
                                                if dp > 1 else None)}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
